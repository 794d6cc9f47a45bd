#include "transfer.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/fs.h>
#include <sys/ioctl.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace tpi {

namespace {

std::string join(const std::string& a, const std::string& b) {
  if (b.empty()) return a;
  if (a.empty()) return b;
  return a.back() == '/' ? a + b : a + "/" + b;
}

int64_t mtime_ns_of(const struct stat& st) {
  return (int64_t)st.st_mtim.tv_sec * 1000000000LL + st.st_mtim.tv_nsec;
}

void walk_rec(const std::string& root, const std::string& rel, const Filter& f,
              std::vector<Entry>& out) {
  std::string dir = join(root, rel);
  DIR* d = opendir(dir.c_str());
  if (!d) throw std::runtime_error("opendir " + dir + ": " + strerror(errno));
  std::vector<std::string> names;
  while (struct dirent* de = readdir(d)) {
    if (!strcmp(de->d_name, ".") || !strcmp(de->d_name, "..")) continue;
    names.emplace_back(de->d_name);
  }
  closedir(d);
  std::sort(names.begin(), names.end());
  std::vector<std::string> subdirs;
  for (auto& name : names) {
    std::string r = rel.empty() ? name : rel + "/" + name;
    struct stat st;
    if (lstat(join(root, r).c_str(), &st)) continue;  // vanished
    if (S_ISLNK(st.st_mode)) continue;
    if (S_ISDIR(st.st_mode)) {
      if (!f.include_dir(r)) continue;
      Entry e;
      e.rel = r;
      e.is_dir = true;
      e.mode = st.st_mode & 07777;
      e.mtime_ns = mtime_ns_of(st);
      out.push_back(e);
      subdirs.push_back(r);
    } else if (S_ISREG(st.st_mode)) {
      if (!f.include_file(r)) continue;
      Entry e;
      e.rel = r;
      e.size = (uint64_t)st.st_size;
      e.mode = st.st_mode & 07777;
      e.mtime_ns = mtime_ns_of(st);
      out.push_back(e);
    }
  }
  for (auto& s : subdirs) walk_rec(root, s, f, out);
}

void mkdirs(const std::string& path, mode_t mode) {
  if (path.empty()) return;
  if (mkdir(path.c_str(), mode) == 0 || errno == EEXIST) return;
  if (errno == ENOENT) {
    auto slash = path.rfind('/');
    if (slash != std::string::npos && slash > 0) mkdirs(path.substr(0, slash), 0755);
    if (mkdir(path.c_str(), mode) == 0 || errno == EEXIST) return;
  }
  throw std::runtime_error("mkdir " + path + ": " + strerror(errno));
}

struct FileJob {
  std::string src, dst, tmp;
  uint64_t size;
  int64_t mtime_ns;
  uint32_t mode;
  int in_fd = -1, out_fd = -1;
  std::atomic<int> pieces_left{0};
  std::atomic<bool> failed{false};
  bool cloned = false;  // FICLONE shared the extents: no pieces to copy
  std::string error;
  std::mutex mu;
};

struct Piece {
  FileJob* job;
  uint64_t off, len;
  uint64_t index;  // piece number within its file
};

bool copy_range(int in, int out, uint64_t off, uint64_t len, std::string& err) {
  loff_t io = (loff_t)off, oo = (loff_t)off;
  uint64_t left = len;
  bool use_cfr = true;
  while (left) {
    ssize_t n = -1;
    if (use_cfr) {
      n = copy_file_range(in, &io, out, &oo, left, 0);
      if (n < 0 && (errno == EXDEV || errno == ENOSYS || errno == EINVAL || errno == EOPNOTSUPP)) {
        use_cfr = false;
        continue;
      }
    } else {
      static thread_local std::unique_ptr<char[]> buf(new char[1 << 20]);
      ssize_t r = pread(in, buf.get(), std::min<uint64_t>(left, 1 << 20), io);
      if (r > 0) {
        ssize_t w = pwrite(out, buf.get(), r, oo);
        if (w != r) r = -1;
        else io += r, oo += r;
      }
      n = r;
    }
    if (n < 0) {
      if (errno == EINTR) continue;
      err = strerror(errno);
      return false;
    }
    if (n == 0) {
      err = "unexpected end of file";
      return false;
    }
    left -= (uint64_t)n;
  }
  return true;
}

void finish_job(FileJob* j) {
  if (j->in_fd >= 0) close(j->in_fd);
  if (j->out_fd >= 0) {
    fchmod(j->out_fd, j->mode);
    struct timespec ts[2];
    ts[0].tv_sec = j->mtime_ns / 1000000000LL;
    ts[0].tv_nsec = j->mtime_ns % 1000000000LL;
    ts[1] = ts[0];
    futimens(j->out_fd, ts);
    close(j->out_fd);
  }
  if (!j->failed && rename(j->tmp.c_str(), j->dst.c_str())) {
    j->failed = true;
    j->error = "rename " + j->dst + ": " + strerror(errno);
  }
  if (j->failed) unlink(j->tmp.c_str());
}

}  // namespace

std::vector<Entry> walk(const std::string& root, const Filter& filter) {
  std::vector<Entry> out;
  struct stat st;
  if (stat(root.c_str(), &st) || !S_ISDIR(st.st_mode))
    throw std::runtime_error("not a directory: " + root);
  walk_rec(root, "", filter, out);
  return out;
}

TransferStats copy_dir(const std::string& src, const std::string& dst, const Filter& filter,
                       int threads, uint64_t piece_bytes) {
  auto t0 = std::chrono::steady_clock::now();
  TransferStats stats;
  std::vector<Entry> entries = walk(src, filter);
  struct stat st;
  mode_t root_mode = 0755;
  if (stat(src.c_str(), &st) == 0) root_mode = st.st_mode & 07777;
  mkdirs(dst, root_mode);
  std::vector<std::unique_ptr<FileJob>> jobs;
  std::vector<Piece> pieces;
  if (piece_bytes == 0) piece_bytes = 256ull << 20;
  for (auto& e : entries) {
    std::string d = join(dst, e.rel);
    if (e.is_dir) {
      mkdirs(d, e.mode ? e.mode : 0755);
      stats.dirs++;
      continue;
    }
    struct stat ds;
    if (stat(d.c_str(), &ds) == 0 && S_ISREG(ds.st_mode) && (uint64_t)ds.st_size == e.size &&
        mtime_ns_of(ds) == e.mtime_ns) {
      stats.skipped++;
      stats.skipped_bytes += e.size;
      continue;
    }
    auto j = std::make_unique<FileJob>();
    j->src = join(src, e.rel);
    j->dst = d;
    j->tmp = d + ".tpi-partial";
    j->size = e.size;
    j->mtime_ns = e.mtime_ns;
    j->mode = e.mode;
    j->in_fd = open(j->src.c_str(), O_RDONLY | O_CLOEXEC);
    if (j->in_fd < 0) throw std::runtime_error("open " + j->src + ": " + strerror(errno));
    j->out_fd = open(j->tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
    if (j->out_fd < 0) {
      close(j->in_fd);
      throw std::runtime_error("open " + j->tmp + ": " + strerror(errno));
    }
    // A copy-on-write clone (XFS reflink, btrfs) shares the extents: the push of a
    // multi-GB workdir becomes a metadata operation.  Elsewhere: parallel byte copies.
    const bool cloned = j->cloned = e.size && ioctl(j->out_fd, FICLONE, j->in_fd) == 0;
    if (!cloned && e.size && ftruncate(j->out_fd, (off_t)e.size)) {
      close(j->in_fd);
      close(j->out_fd);
      throw std::runtime_error("ftruncate " + j->tmp + ": " + strerror(errno));
    }
    uint64_t n = e.size && !cloned ? (e.size + piece_bytes - 1) / piece_bytes : 0;
    if (cloned) stats.cloned++;
    j->pieces_left = (int)n;
    for (uint64_t k = 0; k < n; ++k)
      pieces.push_back(
          {j.get(), k * piece_bytes, std::min(piece_bytes, e.size - k * piece_bytes), k});
    stats.files++;
    stats.bytes += e.size;
    jobs.push_back(std::move(j));
  }
  // Round-robin over files (every file's first piece, then every second piece, ...): writers
  // of one file serialise on its inode lock, so threads working side by side should be on
  // different files.  Within a round, largest pieces first keeps the pool busy to the end.
  std::stable_sort(pieces.begin(), pieces.end(), [](const Piece& a, const Piece& b) {
    return a.index != b.index ? a.index < b.index : a.len > b.len;
  });
  std::atomic<size_t> next{0};
  auto worker = [&] {
    for (;;) {
      size_t i = next.fetch_add(1);
      if (i >= pieces.size()) return;
      Piece& p = pieces[i];
      std::string err;
      if (!p.job->failed && !copy_range(p.job->in_fd, p.job->out_fd, p.off, p.len, err)) {
        std::lock_guard<std::mutex> lk(p.job->mu);
        p.job->failed = true;
        p.job->error = p.job->src + ": " + err;
      }
      if (p.job->pieces_left.fetch_sub(1) == 1) finish_job(p.job);
    }
  };
  int nth = std::max(1, std::min<int>(threads, (int)pieces.size()));
  std::vector<std::thread> pool;
  for (int i = 0; i < nth - 1; ++i) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
  std::string first_error;
  for (auto& j : jobs) {
    if (j->size == 0 || j->cloned) finish_job(j.get());  // no pieces: finish here
    if (j->failed && first_error.empty()) first_error = j->error;
  }
  if (!first_error.empty()) throw std::runtime_error(first_error);
  stats.seconds =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return stats;
}

namespace {

template <class F>
uint64_t pool_over(size_t n, int threads, F&& f) {
  std::atomic<size_t> next{0};
  std::atomic<uint64_t> done{0};
  std::string first_error;
  std::mutex mu;
  auto worker = [&] {
    for (;;) {
      size_t i = next.fetch_add(1);
      if (i >= n) return;
      std::string err;
      uint64_t got = f(i, err);
      if (!err.empty()) {
        std::lock_guard<std::mutex> lk(mu);
        if (first_error.empty()) first_error = err;
      }
      done += got;
    }
  };
  int nth = std::max(1, std::min<int>(threads, (int)n));
  std::vector<std::thread> pool;
  for (int i = 0; i < nth - 1; ++i) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
  if (!first_error.empty()) throw std::runtime_error(first_error);
  return done;
}

// Large pieces are cut into <= kSplit sub-pieces so one big file still spreads over the
// whole thread pool (page-cache -> pinned memcpy is per-thread bound at a few GB/s).
constexpr uint64_t kSplit = 8ull << 20;

std::vector<ReadPiece> split_pieces(const std::vector<ReadPiece>& pieces) {
  std::vector<ReadPiece> out;
  out.reserve(pieces.size());
  for (const ReadPiece& p : pieces) {
    for (uint64_t o = 0; o < p.len || (o == 0 && p.len == 0); o += kSplit) {
      out.push_back({p.path, p.file_off + o, std::min(kSplit, p.len - o), p.dst_off + o});
      if (p.len == 0) break;
    }
  }
  return out;
}

}  // namespace

uint64_t read_pieces(const std::vector<ReadPiece>& in, uint8_t* dst, int threads) {
  const std::vector<ReadPiece> pieces = split_pieces(in);
  return pool_over(pieces.size(), threads, [&](size_t i, std::string& err) -> uint64_t {
    const ReadPiece& p = pieces[i];
    int fd = open(p.path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      err = "open " + p.path + ": " + strerror(errno);
      return 0;
    }
    posix_fadvise(fd, (off_t)p.file_off, (off_t)p.len, POSIX_FADV_SEQUENTIAL);
    uint64_t got = 0;
    while (got < p.len) {
      ssize_t n = pread(fd, dst + p.dst_off + got, p.len - got, (off_t)(p.file_off + got));
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) {
        err = "read " + p.path + ": " + (n < 0 ? strerror(errno) : "short file");
        break;
      }
      got += (uint64_t)n;
    }
    close(fd);
    return got;
  });
}

uint64_t write_pieces(const std::vector<ReadPiece>& in, const uint8_t* src, int threads) {
  const std::vector<ReadPiece> pieces = split_pieces(in);
  return pool_over(pieces.size(), threads, [&](size_t i, std::string& err) -> uint64_t {
    const ReadPiece& p = pieces[i];
    int fd = open(p.path.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
    if (fd < 0) {
      err = "open " + p.path + ": " + strerror(errno);
      return 0;
    }
    uint64_t put = 0;
    while (put < p.len) {
      ssize_t n = pwrite(fd, src + p.dst_off + put, p.len - put, (off_t)(p.file_off + put));
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) {
        err = "write " + p.path + ": " + strerror(errno);
        break;
      }
      put += (uint64_t)n;
    }
    close(fd);
    return put;
  });
}

uint64_t remove_tree(const std::string& path) {
  struct stat st;
  if (lstat(path.c_str(), &st)) return 0;
  uint64_t n = 0;
  if (S_ISDIR(st.st_mode)) {
    // a few passes: a writer that is still appending (a settled supervisor journalling the
    // exit of a released process) may re-create a file between the scan and the rmdir
    for (int pass = 0; pass < 4; ++pass) {
      DIR* d = opendir(path.c_str());
      if (d) {
        std::vector<std::string> names;
        while (struct dirent* de = readdir(d))
          if (strcmp(de->d_name, ".") && strcmp(de->d_name, "..")) names.emplace_back(de->d_name);
        closedir(d);
        for (auto& nme : names) n += remove_tree(join(path, nme));
      }
      if (rmdir(path.c_str()) == 0) {
        ++n;
        break;
      }
      if (errno != ENOTEMPTY && errno != EEXIST) break;
    }
  } else if (unlink(path.c_str()) == 0) {
    ++n;
  }
  return n;
}

}  // namespace tpi
