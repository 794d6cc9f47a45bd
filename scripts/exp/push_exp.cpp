// Round 6 experiment: the workdir push's copy methods on the GPU box's filesystem.
// A 10 GB workdir of 10 files pushes at ~46-60 GB/s with copy_file_range pieces; writers of
// one file serialise on its inode lock, so at most 10 copy at once.  This compares that with
// writes through a shared mapping of the destination (page faults take no inode lock).
// usage: push_exp <src dir with f0..f{n-1}> <dst dir> <files> <threads> <piece MiB> <method>
//   method: cfr (copy_file_range), mmap (pread into a MAP_SHARED destination),
//           mmap_pop (the same after MADV_POPULATE_WRITE of the piece)
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

struct Piece { int f; size_t off, len; };

int main(int argc, char** argv) {
  if (argc != 7) { fprintf(stderr, "usage\n"); return 2; }
  std::string src = argv[1], dst = argv[2];
  int files = atoi(argv[3]), threads = atoi(argv[4]);
  size_t piece = (size_t)atoi(argv[5]) << 20;
  std::string method = argv[6];
  std::vector<int> in(files), out(files);
  std::vector<size_t> size(files);
  std::vector<char*> map(files, nullptr);
  auto t0 = std::chrono::steady_clock::now();
  std::vector<Piece> pieces;
  for (int f = 0; f < files; ++f) {
    std::string s = src + "/f" + std::to_string(f) + ".bin", d = dst + "/f" + std::to_string(f) + ".bin";
    in[f] = open(s.c_str(), O_RDONLY);
    out[f] = open(d.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
    struct stat st;
    if (in[f] < 0 || out[f] < 0 || fstat(in[f], &st)) { perror("open"); return 1; }
    size[f] = st.st_size;
    if (ftruncate(out[f], st.st_size)) { perror("ftruncate"); return 1; }
    if (method != "cfr") {
      map[f] = (char*)mmap(nullptr, size[f], PROT_READ | PROT_WRITE, MAP_SHARED, out[f], 0);
      if (map[f] == MAP_FAILED) { perror("mmap"); return 1; }
    }
  }
  for (size_t off = 0;; off += piece) {  // round-robin over files, as copy_dir does
    bool any = false;
    for (int f = 0; f < files; ++f)
      if (off < size[f]) { pieces.push_back({f, off, std::min(piece, size[f] - off)}); any = true; }
    if (!any) break;
  }
  std::atomic<size_t> next{0};
  std::atomic<int> bad{0};
  auto worker = [&] {
    for (;;) {
      size_t i = next.fetch_add(1);
      if (i >= pieces.size()) return;
      const Piece& p = pieces[i];
      if (method == "cfr") {
        loff_t io = p.off, oo = p.off;
        size_t left = p.len;
        while (left) {
          ssize_t n = copy_file_range(in[p.f], &io, out[p.f], &oo, left, 0);
          if (n <= 0) { bad++; break; }
          left -= n;
        }
      } else {
        char* base = map[p.f] + p.off;
        if (method == "mmap_pop" && madvise(base, p.len, MADV_POPULATE_WRITE)) bad++;
        size_t done = 0;
        while (done < p.len) {
          ssize_t n = pread(in[p.f], base + done, p.len - done, p.off + done);
          if (n <= 0) { bad++; break; }
          done += n;
        }
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) pool.emplace_back(worker);
  for (auto& t : pool) t.join();
  size_t total = 0;
  for (int f = 0; f < files; ++f) {
    if (map[f]) munmap(map[f], size[f]);
    close(in[f]);
    close(out[f]);
    total += size[f];
  }
  double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"method\": \"%s\", \"threads\": %d, \"piece_mib\": %zu, \"bytes\": %zu, \"s\": %.4f, "
         "\"GBps\": %.2f, \"errors\": %d}\n", method.c_str(), threads, piece >> 20, total, s,
         total / s / 1e9, bad.load());
  return bad ? 1 : 0;
}
