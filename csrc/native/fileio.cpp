// Parallel checkpoint file I/O (Checkpointer.persist / load).
//
// The reference persists a task's data as an rclone upload to the bucket and restores it with
// `rclone copy` before the script starts (machine-script.sh.tpl:89,118-124).  Here a checkpoint
// region (host DRAM, pinned) goes to a file on the node and back:
//
//   write_file     threads pwrite disjoint 64 MiB pieces of [src, src + n) into a new file,
//                  then fsync (what a single Python write() + fsync did at 5.6 GB/s).
//   read_stream    reads [offset, offset + n) of a file into memory in chunks, each chunk
//                  split over the threads, and after every chunk release-stores the progress
//                  words of a streamed checkpoint (bytes, then the number of whole tiles, from
//                  the tiles' end offsets): the device restore (tpi_restore_stream) runs
//                  behind the read instead of after it.
#include "fileio.h"

#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

namespace tpi {

namespace {

constexpr uint64_t kPiece = 64ull << 20;

std::string errtext(const char* what, const std::string& path) {
  return std::string(what) + " " + path + ": " + strerror(errno);
}

// Run fn(piece index) for pieces [0, n) on `threads` threads; returns the first error text.
template <class F>
std::string run_pieces(uint64_t n, int threads, F&& fn) {
  std::atomic<uint64_t> next{0};
  std::vector<std::string> errs(std::max(1, threads));
  auto worker = [&](int t) {
    for (uint64_t i; (i = next.fetch_add(1)) < n;) {
      std::string e = fn(i);
      if (!e.empty()) {
        errs[t] = e;
        next.store(n);
        return;
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(worker, t);
  worker(0);
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (!e.empty()) return e;
  return "";
}

}  // namespace

std::string write_file(const std::string& path, const void* src, uint64_t n, int threads,
                       bool sync) {
  int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
  if (fd < 0) return errtext("open", path);
  std::string err;
  if (ftruncate(fd, (off_t)n) != 0) err = errtext("ftruncate", path);
  if (err.empty()) {
    const uint8_t* base = (const uint8_t*)src;
    err = run_pieces((n + kPiece - 1) / kPiece, threads, [&](uint64_t i) -> std::string {
      const uint64_t lo = i * kPiece, hi = std::min(n, lo + kPiece);
      for (uint64_t at = lo; at < hi;) {
        ssize_t w = pwrite(fd, base + at, hi - at, (off_t)at);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) return errtext("write", path);
        at += (uint64_t)w;
      }
      return "";
    });
  }
  if (err.empty() && sync && fsync(fd) != 0) err = errtext("fsync", path);
  close(fd);
  return err;
}

std::string read_stream(const std::string& path, void* dst, uint64_t offset, uint64_t n,
                        int threads, uint64_t chunk, uint64_t* words, const uint64_t* tile_ends,
                        uint64_t ntiles) {
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return errtext("open", path);
  posix_fadvise(fd, (off_t)offset, (off_t)n, POSIX_FADV_SEQUENTIAL);
  uint8_t* base = (uint8_t*)dst;
  chunk = std::max<uint64_t>(chunk, 4096);
  std::string err;
  uint64_t tiles = 0;
  for (uint64_t a = 0; a < n && err.empty(); a += chunk) {
    const uint64_t b = std::min(n, a + chunk);
    const uint64_t per = ((b - a + threads - 1) / std::max(1, threads) + 4095) / 4096 * 4096;
    err = run_pieces((b - a + per - 1) / per, threads, [&](uint64_t i) -> std::string {
      const uint64_t lo = a + i * per, hi = std::min(b, lo + per);
      for (uint64_t at = lo; at < hi;) {
        ssize_t r = pread(fd, base + at, hi - at, (off_t)(offset + at));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return r < 0 ? errtext("read", path) : "read " + path + ": file truncated";
        at += (uint64_t)r;
      }
      return "";
    });
    if (err.empty() && words) {
      while (tiles < ntiles && tile_ends[tiles] <= b) ++tiles;
      __atomic_store_n(&words[1], b, __ATOMIC_RELEASE);
      __atomic_store_n(&words[0], tiles, __ATOMIC_RELEASE);
    }
  }
  close(fd);
  return err;
}

}  // namespace tpi
