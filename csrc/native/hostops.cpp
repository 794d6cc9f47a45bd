// Host (CPU) implementations of the data-plane primitives: CRC32C tiles (SSE4.2 crc32
// instruction, 3-way interleaved), striped XXH64 shard hashes and pack/unpack of CPU tensors.
// They define the on-disk/in-memory formats bit-for-bit identically to the HIP kernels in
// csrc/hip/kernels.hip (tests compare both) and serve the `local` (CPU) backend.
#include "hostops.h"

#include <fcntl.h>
#include <nmmintrin.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <stdexcept>
#include <thread>
#include <vector>

#include "../common/crc32c.h"
#include "../common/tpz.h"
#include "../common/xxh64.h"

namespace tpi {

namespace {

const tpi_crc_tables& tables() {
  static tpi_crc_tables t = [] {
    tpi_crc_tables x;
    tpi_crc_tables_init(&x);
    return x;
  }();
  return t;
}

uint32_t crc_update_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n && ((uintptr_t)p & 7)) {
    c = _mm_crc32_u8((uint32_t)c, *p++);
    --n;
  }
  // Three independent streams hide the 3-cycle latency of crc32q; recombine with shifts.
  const size_t block = 8192;
  while (n >= 3 * block) {
    uint64_t c1 = 0, c2 = 0;
    const uint8_t* p1 = p + block;
    const uint8_t* p2 = p + 2 * block;
    for (size_t i = 0; i < block; i += 8) {
      uint64_t a, b, d;
      memcpy(&a, p + i, 8);
      memcpy(&b, p1 + i, 8);
      memcpy(&d, p2 + i, 8);
      c = _mm_crc32_u64(c, a);
      c1 = _mm_crc32_u64(c1, b);
      c2 = _mm_crc32_u64(c2, d);
    }
    const uint32_t k = tpi_x8nmodp(block, tables().x2n);
    c = tpi_multmodp(k, tpi_multmodp(k, (uint32_t)c) ^ (uint32_t)c1) ^ (uint32_t)c2;
    p += 3 * block;
    n -= 3 * block;
  }
  while (n >= 8) {
    uint64_t a;
    memcpy(&a, p, 8);
    c = _mm_crc32_u64(c, a);
    p += 8;
    n -= 8;
  }
  while (n--) c = _mm_crc32_u8((uint32_t)c, *p++);
  return (uint32_t)c;
}

template <class F>
void parallel_for(uint64_t n, int threads, F&& f) {
  if (n == 0) return;
  int nth = (int)std::max<uint64_t>(1, std::min<uint64_t>(threads, n));
  std::atomic<uint64_t> next{0};
  auto worker = [&] {
    for (;;) {
      uint64_t i = next.fetch_add(1);
      if (i >= n) return;
      f(i);
    }
  };
  std::vector<std::thread> pool;
  for (int i = 0; i < nth - 1; ++i) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
}

}  // namespace

uint32_t crc32c(const void* data, size_t n, uint32_t crc) {
  return ~crc_update_hw(~crc, (const uint8_t*)data, n);
}

uint32_t crc32c_combine(uint32_t a, uint32_t b, uint64_t len_b) {
  return tpi_crc32c_combine(a, b, len_b, tables().x2n);
}

uint32_t crc32c_combine_tiles(const uint32_t* crcs, uint64_t ntiles, uint64_t tile,
                              uint64_t total) {
  if (ntiles == 0) return 0;
  const uint32_t k_full = tpi_x8nmodp(tile, tables().x2n);
  uint32_t crc = crcs[0];
  for (uint64_t t = 1; t < ntiles; ++t) {
    const uint64_t len = std::min(tile, total - t * tile);
    const uint32_t k = len == tile ? k_full : tpi_x8nmodp(len, tables().x2n);
    crc = tpi_multmodp(k, crc) ^ crcs[t];
  }
  return crc;
}

void crc32c_tiles(const void* data, uint64_t n, uint64_t tile, uint32_t* out, int threads) {
  if (tile == 0) throw std::invalid_argument("tile must be positive");
  const uint8_t* p = (const uint8_t*)data;
  parallel_for((n + tile - 1) / tile, threads, [&](uint64_t t) {
    out[t] = crc32c(p + t * tile, std::min(tile, n - t * tile), 0);
  });
}

void shard_hash(const void* data, uint64_t n, uint64_t shard, uint64_t seed, uint64_t* out,
                int threads) {
  if (shard == 0) throw std::invalid_argument("shard must be positive");
  const uint8_t* p = (const uint8_t*)data;
  parallel_for((n + shard - 1) / shard, threads, [&](uint64_t s) {
    out[s] = tpi_shard_hash_host(p + s * shard, std::min(shard, n - s * shard), seed);
  });
}

namespace {

uint64_t strided_offset(const tpi_seg& s, uint64_t e) {
  uint64_t off = 0;
  for (int d = s.ndim - 1; d >= 0; --d) {
    uint64_t sz = (uint64_t)s.sizes[d];
    off += (e % sz) * (uint64_t)s.strides[d];
    e /= sz;
  }
  return off;
}

void copy_segment(const tpi_seg& s, uint8_t* stream, uint64_t lo, uint64_t hi, bool pack) {
  // Bytes [lo, hi) of the payload of `s` (payload-relative).
  if (s.kind == 0) {
    uint8_t* t = (uint8_t*)s.ptr;
    if (pack) memcpy(stream + s.off + lo, t + lo, hi - lo);
    else memcpy(t + lo, stream + s.off + lo, hi - lo);
    return;
  }
  for (uint64_t q = lo; q < hi;) {
    uint64_t e = q / s.elem, within = q % s.elem;
    uint64_t take = std::min<uint64_t>(s.elem - within, hi - q);
    uint8_t* t = (uint8_t*)s.ptr + strided_offset(s, e) * s.elem + within;
    if (pack) memcpy(stream + s.off + q, t, take);
    else memcpy(t, stream + s.off + q, take);
    q += take;
  }
}

// Process tile t: pack/unpack the payload bytes that fall inside it, zero the padding.
void process_tile(const tpi_seg* segs, int n, uint8_t* stream, uint64_t total, uint64_t tile,
                  uint64_t t, bool pack) {
  const uint64_t lo = t * tile, hi = std::min(total, lo + tile);
  int i = 0, a = 0, b = n - 1;
  while (a < b) {  // largest i with off <= lo
    int m = (a + b + 1) / 2;
    if (segs[m].off <= lo) a = m; else b = m - 1;
  }
  i = a;
  uint64_t pos = lo;
  for (; i < n && pos < hi; ++i) {
    const tpi_seg& s = segs[i];
    if (s.off >= hi) break;
    if (pack && s.off > pos) memset(stream + pos, 0, s.off - pos);
    uint64_t a0 = std::max(pos, s.off), a1 = std::min(hi, s.off + s.nbytes);
    if (a1 > a0) copy_segment(s, stream, a0 - s.off, a1 - s.off, pack);
    pos = std::max(pos, std::max(a1, s.off));
  }
  if (pack && pos < hi) memset(stream + pos, 0, hi - pos);
}

}  // namespace

void pack(const tpi_seg* segs, int n, uint64_t total, void* stream, uint64_t tile,
          uint32_t* crcs, int threads) {
  uint8_t* st = (uint8_t*)stream;
  parallel_for((total + tile - 1) / tile, threads, [&](uint64_t t) {
    process_tile(segs, n, st, total, tile, t, true);
    const uint64_t lo = t * tile;
    crcs[t] = crc32c(st + lo, std::min(tile, total - lo), 0);
  });
}

uint64_t unpack(const tpi_seg* segs, int n, uint64_t total, const void* stream, uint64_t tile,
                const uint32_t* crcs, int threads, int64_t* first_bad) {
  uint8_t* st = (uint8_t*)stream;
  std::atomic<uint64_t> bad{0};
  std::atomic<int64_t> first{INT64_MAX};
  parallel_for((total + tile - 1) / tile, threads, [&](uint64_t t) {
    const uint64_t lo = t * tile;
    if (crc32c(st + lo, std::min(tile, total - lo), 0) != crcs[t]) {
      bad++;
      int64_t cur = first.load();
      while ((int64_t)t < cur && !first.compare_exchange_weak(cur, (int64_t)t)) {
      }
    }
    process_tile(segs, n, st, total, tile, t, false);
  });
  *first_bad = bad ? first.load() : -1;
  return bad;
}

int64_t resident_bytes(const char* path, uint64_t* size, int* tmpfs) {
  *size = 0;
  *tmpfs = 0;
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  struct stat st;
  struct statfs sf;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return -1;
  }
  if (fstatfs(fd, &sf) == 0) *tmpfs = sf.f_type == 0x01021994 /* TMPFS_MAGIC */;
  *size = (uint64_t)st.st_size;
  if (st.st_size == 0) {
    close(fd);
    return 0;
  }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return -1;
  const long page = sysconf(_SC_PAGESIZE);
  const uint64_t pages = ((uint64_t)st.st_size + page - 1) / page;
  std::vector<unsigned char> vec(pages);
  int64_t resident = -1;
  if (mincore(p, (size_t)st.st_size, vec.data()) == 0) {
    resident = 0;
    for (unsigned char v : vec) resident += (v & 1);
    resident *= page;
    if (resident > st.st_size) resident = st.st_size;
  }
  munmap(p, (size_t)st.st_size);
  return resident;
}

uint64_t tpz_encode_stream(const void* src, uint64_t total, uint64_t tile, void* dst,
                           uint32_t* csizes, int threads) {
  // Same two passes as the GPU: headers + sizes, then blobs written at their offsets.
  const uint64_t ntiles = (total + tile - 1) / tile;
  const uint8_t* s = (const uint8_t*)src;
  std::vector<tpz_plane> hdr(ntiles * 4);
  std::vector<uint8_t> lens(ntiles * 64);  // HUF code lengths, 16 per plane
  auto lens_of = [&](uint64_t t) { return (uint8_t(*)[16])(lens.data() + t * 64); };
  parallel_for(ntiles, threads, [&](uint64_t t) {
    const uint64_t lo = t * tile;
    csizes[t] = (uint32_t)tpz_analyze_tile(s + lo, std::min(tile, total - lo), &hdr[t * 4],
                                           lens_of(t));
  });
  std::vector<uint64_t> off(ntiles + 1, 0);
  for (uint64_t t = 0; t < ntiles; ++t) off[t + 1] = off[t] + csizes[t];
  parallel_for(ntiles, threads, [&](uint64_t t) {
    const uint64_t lo = t * tile;
    tpz_emit_tile(s + lo, std::min(tile, total - lo), &hdr[t * 4], lens_of(t),
                  (uint8_t*)dst + off[t]);
  });
  return off[ntiles];
}

int64_t tpz_decode_stream(const void* src, const uint32_t* csizes, uint64_t total, uint64_t tile,
                          void* dst, int threads) {
  const uint64_t ntiles = (total + tile - 1) / tile;
  std::vector<uint64_t> off(ntiles + 1, 0);
  for (uint64_t t = 0; t < ntiles; ++t) off[t + 1] = off[t] + csizes[t];
  std::atomic<int64_t> first{INT64_MAX};
  parallel_for(ntiles, threads, [&](uint64_t t) {
    const uint64_t lo = t * tile, len = std::min(tile, total - lo);
    if (tpz_decode_tile((const uint8_t*)src + off[t], csizes[t], len, (uint8_t*)dst + lo) !=
        csizes[t]) {
      memset((uint8_t*)dst + lo, 0, len);
      int64_t cur = first.load();
      while ((int64_t)t < cur && !first.compare_exchange_weak(cur, (int64_t)t)) {
      }
    }
  });
  return first.load() == INT64_MAX ? -1 : first.load();
}

}  // namespace tpi
