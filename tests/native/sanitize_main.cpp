// Host-code sanitizer harness: built by tests/test_sanitizers.py with
// -fsanitize=address,undefined -fno-sanitize-recover=all together with the production
// sources in csrc/native, then run.  Exits non-zero on the first failed check; the
// sanitizers abort on any memory/UB error.
//
// Covers: glob/filter parsing and matching (incl. malformed patterns), walk/copy_dir/
// remove_tree on a scratch tree, CRC32C tiles + combine, shard hash, pack/unpack of
// contiguous and strided segments, and the TPZ1 codec: round trips on float-like data plus
// a decoder fuzz over randomly corrupted and truncated blobs (checkpoint files are untrusted
// input), the parallel checkpoint file I/O and the step-boundary agreement block.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../csrc/common/tpz.h"
#include "../../csrc/native/ctl.h"
#include "../../csrc/native/fileio.h"
#include "../../csrc/native/filter.h"
#include "../../csrc/native/hostops.h"
#include "../../csrc/native/transfer.h"

static int g_fail = 0;
#define CHECK(cond)                                                  \
  do {                                                               \
    if (!(cond)) {                                                   \
      fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      g_fail = 1;                                                    \
    }                                                                \
  } while (0)

static void write_file(const std::string& path, size_t n, unsigned seed) {
  FILE* f = fopen(path.c_str(), "wb");
  std::mt19937 rng(seed);
  for (size_t i = 0; i < n; ++i) fputc((int)(rng() & 0xff), f);
  fclose(f);
}

static void test_filters() {
  tpi::Filter f;
  f.add_rule("- /main.tf");
  f.add_rule("- /.terraform**");
  f.add_rule("- *.tmp");
  f.add_rule("+ /keep/**");
  f.add_rule("- {a,b}[0-9]?.bin");
  CHECK(!f.include_file("main.tf"));
  CHECK(f.include_file("sub/main.tf"));
  CHECK(!f.include_file(".terraform/x/y"));
  CHECK(!f.include_file("deep/dir/x.tmp"));
  CHECK(f.include_file("keep/z.tmp") == false);  // first match wins: *.tmp
  CHECK(!f.include_file("a1x.bin"));
  CHECK(f.include_file("c1x.bin"));
  const char* bad[] = {"[", "a[b", "{a,b", "\\", "[z-a]", "**{", ""};
  for (const char* b : bad) {
    try {
      tpi::Glob g(b);
      (void)g.match("anything/at/all");
    } catch (const std::invalid_argument&) {
    }
  }
  std::mt19937 rng(1);
  const char alphabet[] = "ab*?/[]{},\\-!^.";
  for (int i = 0; i < 3000; ++i) {  // random patterns never crash
    std::string pat, path;
    for (int j = rng() % 12; j > 0; --j) pat += alphabet[rng() % (sizeof(alphabet) - 1)];
    for (int j = rng() % 16; j > 0; --j) path += "ab/c."[rng() % 5];
    try {
      tpi::Glob g(pat);
      (void)g.match(path);
    } catch (const std::invalid_argument&) {
    }
  }
}

static void test_transfer(const std::string& scratch) {
  const std::string src = scratch + "/src", dst = scratch + "/dst";
  mkdir(src.c_str(), 0755);
  mkdir((src + "/d1").c_str(), 0755);
  mkdir((src + "/d1/d2").c_str(), 0755);
  mkdir((src + "/empty").c_str(), 0755);
  write_file(src + "/a.bin", 100000, 1);
  write_file(src + "/d1/b.bin", 3 << 20, 2);
  write_file(src + "/d1/d2/c.tmp", 10, 3);
  write_file(src + "/zero", 0, 4);
  tpi::Filter f;
  f.add_rule("- *.tmp");
  auto ents = tpi::walk(src, f);
  size_t files = 0;
  for (auto& e : ents) files += !e.is_dir;
  CHECK(files == 3);
  auto st = tpi::copy_dir(src, dst, f, 4, 1 << 20);  // small pieces: multi-piece files
  CHECK(st.files == 3);
  auto again = tpi::copy_dir(src, dst, f, 4, 1 << 20);
  CHECK(again.files == 0 && again.skipped == 3);
  std::vector<tpi::ReadPiece> pieces = {{src + "/d1/b.bin", 1000, 5000, 0},
                                        {src + "/a.bin", 0, 100000, 5000}};
  std::vector<uint8_t> buf(105000);
  CHECK(tpi::read_pieces(pieces, buf.data(), 2) == 105000);
  CHECK(tpi::remove_tree(dst) > 0);
  CHECK(tpi::remove_tree(dst) == 0);
}

static std::vector<uint8_t> float_like(size_t n, unsigned seed) {
  std::mt19937 rng(seed);
  std::normal_distribution<float> nd(0.f, 1e-3f);
  std::vector<uint8_t> out(n);
  size_t i = 0;
  for (; i + 4 <= n / 2; i += 4) {
    float v = nd(rng);
    memcpy(&out[i], &v, 4);
  }
  for (; i < n; ++i) out[i] = (uint8_t)(rng() % 3);  // low-entropy tail
  return out;
}

static void test_hostops() {
  std::vector<uint8_t> data = float_like((1 << 20) + 4096 * 3 + 16, 5);
  const uint64_t tile = 65536, ntiles = (data.size() + tile - 1) / tile;
  std::vector<uint32_t> crcs(ntiles);
  tpi::crc32c_tiles(data.data(), data.size(), tile, crcs.data(), 4);
  CHECK(tpi::crc32c_combine_tiles(crcs.data(), ntiles, tile, data.size()) ==
        tpi::crc32c(data.data(), data.size()));
  std::vector<uint64_t> sh((data.size() + 8191) / 8192);
  tpi::shard_hash(data.data(), data.size(), 8192, 7, sh.data(), 3);

  // pack/unpack: one contiguous + one transposed (strided) tensor
  std::vector<float> a(1000), b(33 * 17), a2(1000), b2(33 * 17);
  for (size_t i = 0; i < a.size(); ++i) a[i] = (float)i;
  for (size_t i = 0; i < b.size(); ++i) b[i] = (float)(i * 3);
  tpi_seg segs[2];
  memset(segs, 0, sizeof(segs));
  segs[0].ptr = (uint64_t)a.data();
  segs[0].off = 0;
  segs[0].nbytes = 4000;
  segs[1].ptr = (uint64_t)b.data();
  segs[1].off = 4096;
  segs[1].nbytes = b.size() * 4;
  segs[1].kind = 1;
  segs[1].elem = 4;
  segs[1].ndim = 2;
  segs[1].sizes[0] = 17;
  segs[1].sizes[1] = 33;
  segs[1].strides[0] = 1;
  segs[1].strides[1] = 17;
  const uint64_t total = 4096 + ((b.size() * 4 + 255) / 256) * 256;
  std::vector<uint8_t> stream(total);
  std::vector<uint32_t> pcrc((total + 4095) / 4096);
  tpi::pack(segs, 2, total, stream.data(), 4096, pcrc.data(), 2);
  segs[0].ptr = (uint64_t)a2.data();
  segs[1].ptr = (uint64_t)b2.data();
  int64_t first = 0;
  CHECK(tpi::unpack(segs, 2, total, stream.data(), 4096, pcrc.data(), 2, &first) == 0);
  CHECK(first == -1 && a == a2 && b == b2);
  stream[5000] ^= 1;
  CHECK(tpi::unpack(segs, 2, total, stream.data(), 4096, pcrc.data(), 2, &first) == 1);
}

static void test_codec() {
  std::mt19937 rng(9);
  for (uint64_t len : {16ull, 144ull, 4096ull, 4096ull * 3 + 48, 65536ull, 1ull << 20}) {
    std::vector<uint8_t> raw = float_like(len, (unsigned)len);
    std::vector<uint8_t> blob(tpz_bound(len)), back(len);
    const uint64_t n = tpz_encode_tile(raw.data(), len, blob.data());
    CHECK(n <= tpz_bound(len) && n % 16 == 0);
    CHECK(tpz_decode_tile(blob.data(), n, len, back.data()) == n);
    CHECK(back == raw);
    // fuzz: flip bytes / truncate; decoder must stay in bounds (ASan) and never hang
    for (int it = 0; it < 400; ++it) {
      std::vector<uint8_t> bad(blob.begin(), blob.begin() + n);
      const int flips = 1 + (int)(rng() % 4);
      for (int f = 0; f < flips; ++f) bad[rng() % n] ^= (uint8_t)(1 + rng() % 255);
      uint64_t avail = (it % 5 == 0) ? rng() % (n + 1) : n;
      bad.resize(avail);
      std::vector<uint8_t> out(len);
      (void)tpz_decode_tile(bad.data(), avail, len, out.data());
    }
  }
  // stream API with a malformed middle tile
  std::vector<uint8_t> raw = float_like(8 * 4096, 3);
  std::vector<uint8_t> enc(8 * tpz_bound(4096)), dec(raw.size());
  std::vector<uint32_t> sizes(8);
  const uint64_t used = tpi::tpz_encode_stream(raw.data(), raw.size(), 4096, enc.data(),
                                               sizes.data(), 3);
  CHECK(tpi::tpz_decode_stream(enc.data(), sizes.data(), raw.size(), 4096, dec.data(), 3) == -1);
  CHECK(dec == raw);
  enc[sizes[0] + sizes[1] + sizes[2]] = 0xEE;  // tile 3 header: invalid mode
  CHECK(tpi::tpz_decode_stream(enc.data(), sizes.data(), raw.size(), 4096, dec.data(), 3) == 3);
  (void)used;
}

// Checkpoint file I/O: parallel write + streamed read with progress words, odd sizes,
// more threads than pieces, a truncated file and a missing one.
static void test_fileio(const std::string& scratch) {
  for (uint64_t n : {0ull, 1ull, 4095ull, (3ull << 20) + 17}) {
    std::vector<uint8_t> src = float_like(n + 16, (unsigned)n);
    src.resize(n);
    const std::string path = scratch + "/ckpt-" + std::to_string(n);
    CHECK(tpi::write_file(path, src.data(), n, 5, true).empty());
    std::vector<uint8_t> back(n + 1, 0xAB);
    std::vector<uint64_t> tile_ends;
    for (uint64_t e = 65536; e < n; e += 65536) tile_ends.push_back(e);
    tile_ends.push_back(n);
    uint64_t words[2] = {0, 0};
    CHECK(tpi::read_stream(path, back.data(), 0, n, 3, 1 << 20, words, tile_ends.data(),
                           tile_ends.size()).empty());
    CHECK(std::equal(src.begin(), src.end(), back.begin()));
    CHECK(back[n] == 0xAB);  // nothing past the end
    if (n) CHECK(words[1] == n && words[0] == tile_ends.size());
    // offset read of the tail, zero threads (clamped to one)
    if (n > 100) {
      std::vector<uint8_t> tail(n - 100);
      CHECK(tpi::read_stream(path, tail.data(), 100, n - 100, 0, 4096, nullptr, nullptr, 0)
                .empty());
      CHECK(std::equal(tail.begin(), tail.end(), src.begin() + 100));
    }
    // asking for more than the file holds is an error, not an overrun
    std::vector<uint8_t> over(n + 8192);
    CHECK(!tpi::read_stream(path, over.data(), 0, n + 8192, 4, 4096, nullptr, nullptr, 0)
               .empty());
  }
  std::vector<uint8_t> buf(64);
  CHECK(!tpi::read_stream(scratch + "/missing", buf.data(), 0, 64, 2, 4096, nullptr, nullptr, 0)
             .empty());
  CHECK(!tpi::write_file(scratch + "/no/such/dir/f", buf.data(), 64, 2, false).empty());
}

// Step-boundary agreement, single thread: the targets a proposer chooses (see ctl.h).
static void test_ctl() {
  const int world = 3;
  std::vector<uint64_t> mem(tpi::ctl::bytes(world) / 8);
  void* b = mem.data();
  CHECK(!tpi::ctl::valid(b, world));
  tpi::ctl::init(b, world);
  CHECK(tpi::ctl::valid(b, world) && !tpi::ctl::valid(b, world + 1));
  uint64_t pre = 1, per = 1;
  tpi::ctl::arrive(b, 0, 5, &pre, &per);
  CHECK(pre == 0 && per == 0);
  tpi::ctl::arrive(b, 1, 7, &pre, &per);
  tpi::ctl::arrive(b, 2, 6, &pre, &per);
  // rank 0 (at 5) proposes: past everyone else's published boundary
  CHECK(tpi::ctl::propose_preempt(b, world, 0) == 8);
  CHECK(tpi::ctl::propose_preempt(b, world, 2) == 8);  // chosen once
  tpi::ctl::arrive(b, 1, 8, &pre, &per);
  CHECK(pre == 8);
  // periodic: rank 0 proposes only when everybody passed the previous target
  CHECK(tpi::ctl::propose_periodic(b, world, 0) == 9);
  CHECK(tpi::ctl::propose_periodic(b, world, 0) == 0);  // rank 0 itself is at 5
  tpi::ctl::arrive(b, 0, 10, &pre, &per);
  tpi::ctl::arrive(b, 1, 10, &pre, &per);
  tpi::ctl::arrive(b, 2, 10, &pre, &per);
  CHECK(per == 9);
  CHECK(tpi::ctl::propose_periodic(b, world, 0) == 11);
  CHECK(tpi::ctl::ordinal_of(b, 2) == 10);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <scratch-dir>\n", argv[0]);
    return 2;
  }
  test_filters();
  test_transfer(argv[1]);
  test_hostops();
  test_codec();
  test_fileio(argv[1]);
  test_ctl();
  if (g_fail) return 1;
  printf("sanitize harness ok\n");
  return 0;
}
