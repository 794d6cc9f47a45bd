// tpi-stager: the per-task workdir data plane on a node (one process per task).
//
// The reference restores the task directory on every machine before the user script starts
// (`rclone copy $RCLONE_REMOTE/data /opt/task/directory`, machine-script.sh.tpl:89; every one
// of the `parallelism` VMs of resource_auto_scaling_group.go:70 does it independently over its
// own link) and re-syncs it every 10 s when the newest mtime changed (tpl:118-124).  On an
// MI355X node the supervisor starts this process before the ranks instead.  It
//
//  1. allocates the workdir image (files at 4 KiB-aligned offsets, runtime/stage.py lays it
//     out) in HBM on every rank's GPU;
//  2. loads it from the page cache: with `method` "sharded" (default) GPU i reads only the i-th
//     1/N of the image over its own PCIe link (libtpi_hip loader: NUMA-local pinned ring, pread
//     workers overlapping the H2D copies), "broadcast" loads everything into GPU 0,
//     "independent" loads everything into every GPU (the reference's pattern, the baseline);
//  3. fans out over xGMI with the task communicator: one in-place ncclAllGather ("sharded") or
//     ncclBroadcast from GPU 0 ("broadcast");
//  4. verifies every copy with the shard-hash kernel (all GPUs' digests must agree);
//  5. publishes the HIP IPC handle of each copy in the manifest, prints "staged" on stdout
//     (the supervisor then starts the ranks with TPI_HBM_WORKDIR=<manifest>), and stays alive
//     holding the images (a respawned rank re-attaches without restaging);
//  6. every `sync_interval` s (and on SIGUSR1, and at SIGTERM) hashes rank 0's copy on device,
//     and writes only the shards that changed back into the task's files (journalled as
//     `workdir-sync` events).
//
// `"host": true` keeps the images in /dev/shm files instead of HBM (CPU rehearsal; same
// loader, layout, fan-out schedule and sync logic).
//
//   tpi-stager <stage.json>
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../common/xxh64.h"
#include "../hip/tpi_hip.h"
#include "../supervisor/json.h"

using tpi::json::quote;
using tpi::json::Value;

namespace {

double now() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

[[noreturn]] void die(const std::string& what) {
  fprintf(stderr, "tpi-stager: %s\n", what.c_str());
  fflush(stderr);
  _exit(1);
}

void check(int rc, const char* what) {
  if (rc != 0) die(std::string(what) + ": " + tpi_last_error());
}

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) die(std::string(what) + ": " + hipGetErrorString(e));
}

std::string read_file(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) die("cannot read " + path);
  std::stringstream ss;
  ss << in.rdbuf();
  return ss.str();
}

bool atomic_write(const std::string& path, const std::string& data) {
  const std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "w");
  if (!f) return false;
  fwrite(data.data(), 1, data.size(), f);
  fclose(f);
  return rename(tmp.c_str(), path.c_str()) == 0;
}

std::string hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = d[p[i] >> 4];
    s[2 * i + 1] = d[p[i] & 15];
  }
  return s;
}

struct Spec {
  std::string root, manifest, events, method = "sharded", shm_prefix;
  std::vector<std::string> paths;  // absolute
  std::vector<std::string> rel;
  std::vector<tpi_file> files;
  uint64_t total = 0, chunk = 64ull << 20, shard_bytes = 1ull << 20;
  int nbuf = 4, threads = 16;
  std::vector<int> devices, numa;
  double sync_interval = 10;
  bool writeback = true, host = false, verify = true;
};

Spec load_spec(const std::string& path) {
  Value v = tpi::json::parse(read_file(path));
  Spec s;
  s.root = v["root"].str();
  s.manifest = v["manifest"].str();
  s.events = v["events"].str();
  s.method = v["method"].str("sharded");
  s.total = (uint64_t)v["total"].num(0);
  s.chunk = (uint64_t)v["chunk_bytes"].num((double)s.chunk);
  s.shard_bytes = (uint64_t)v["shard_bytes"].num((double)s.shard_bytes);
  s.nbuf = (int)v["nbuf"].num(4);
  s.threads = (int)v["threads"].num(16);
  s.sync_interval = v["sync_interval"].num(10);
  s.writeback = v["writeback"].boolean(true);
  s.host = v["host"].boolean(false);
  s.verify = v["verify"].boolean(true);
  s.shm_prefix = v["shm_prefix"].str("/dev/shm/tpi-stage");
  for (auto& d : v["devices"].a) s.devices.push_back((int)d.num(0));
  for (auto& n : v["numa"].a) s.numa.push_back((int)n.num(-1));
  s.numa.resize(s.devices.size(), -1);
  for (auto& f : v["files"].a) {
    s.rel.push_back(f.a.at(0).str());
    s.paths.push_back(s.root + "/" + f.a.at(0).str());
  }
  size_t i = 0;
  for (auto& f : v["files"].a) {
    s.files.push_back({s.paths[i].c_str(), (uint64_t)f.a.at(1).num(0), (uint64_t)f.a.at(2).num(0)});
    ++i;
  }
  const size_t n = s.devices.size();
  if (n == 0) die("spec names no devices");
  if (s.manifest.empty()) die("spec names no manifest");
  if (s.total % (4096 * n)) die("image size must be a multiple of 4096 x ranks");
  for (size_t k = 0; k < s.files.size(); ++k) {
    if (s.files[k].offset + s.files[k].size > s.total) die("file beyond the image: " + s.rel[k]);
    if (k && s.files[k].offset < s.files[k - 1].offset + s.files[k - 1].size)
      die("files overlap or are unsorted");
  }
  if (s.method != "sharded" && s.method != "broadcast" && s.method != "independent")
    die("unknown method " + s.method);
  return s;
}

void event(const Spec& s, const std::string& code, const std::vector<std::string>& desc) {
  if (s.events.empty()) return;
  std::string line = "{\"time\": " + std::to_string(now()) + ", \"code\": " + quote(code) +
                     ", \"description\": [";
  for (size_t i = 0; i < desc.size(); ++i) line += (i ? ", " : "") + quote(desc[i]);
  line += "]}\n";
  int fd = open(s.events.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  if (fd >= 0) {
    ssize_t w = write(fd, line.data(), line.size());
    (void)w;
    close(fd);
  }
}

class Stager {
 public:
  explicit Stager(Spec s) : s_(std::move(s)), n_((int)s_.devices.size()) {}

  void stage() {
    auto t0 = std::chrono::steady_clock::now();
    allocate();
    alloc_ms_ = ms_since(t0);
    load();
    fanout();
    verify();
    publish();
  }

  // Digest every rank's copy and write the shards that changed since the last sync back to
  // the files, each from the rank that changed it (the reference's 10 s loop syncs each
  // machine's own workdir, tpl:118-124).  A shard two ranks changed differently is written
  // from the lowest of them and reported as a conflict.  Returns the number of dirty shards.
  uint64_t sync(const char* why) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::vector<uint64_t>> cur(n_);
    {
      std::vector<std::thread> th;
      for (int i = 0; i < n_; ++i) th.emplace_back([&, i] { cur[i] = digests(i); });
      for (auto& t : th) t.join();
    }
    std::vector<std::vector<uint64_t>> ranges(n_);
    uint64_t dirty = 0, conflicts = 0;
    std::vector<uint64_t> per_rank(n_, 0);
    const uint64_t nshards = cur[0].size();
    for (uint64_t k = 0; k < nshards; ++k) {
      int writer = -1;
      for (int i = 0; i < n_; ++i) {
        if (k < bases_[i].size() && cur[i][k] == bases_[i][k]) continue;
        if (writer < 0) writer = i;
        else if (cur[i][k] != cur[writer][k]) ++conflicts;
      }
      if (writer < 0) continue;
      ++dirty;
      ++per_rank[writer];
      const uint64_t lo = k * s_.shard_bytes, hi = std::min(s_.total, lo + s_.shard_bytes);
      auto& r = ranges[writer];
      if (!r.empty() && r.back() == lo) r.back() = hi;
      else {
        r.push_back(lo);
        r.push_back(hi);
      }
    }
    std::vector<tpi_stats> st(n_);
    if (dirty && s_.writeback) {
      std::vector<std::thread> th;
      std::vector<std::string> errs(n_);
      for (int i = 0; i < n_; ++i)
        if (!ranges[i].empty())
          th.emplace_back([&, i] {
            st[i] = tpi_stats{};
            if (tpi_loader_store(loaders_[i], s_.files.data(), s_.files.size(), ranges[i].data(),
                                 ranges[i].size() / 2, image_[i], &st[i]))
              errs[i] = tpi_last_error();
          });
      for (auto& t : th) t.join();
      for (auto& e : errs)
        if (!e.empty()) die("write-back: " + e);
    }
    bases_ = cur;
    uint64_t bytes = 0;
    for (auto& x : st) bytes += x.bytes;
    std::string who;
    for (int i = 0; i < n_; ++i)
      if (per_rank[i]) who += (who.empty() ? "" : ",") + std::to_string(i) + ":" +
                              std::to_string(per_rank[i]);
    event(s_, "workdir-sync", {why, "dirty_shards " + std::to_string(dirty),
                               "bytes " + std::to_string(bytes),
                               "ranks " + (who.empty() ? std::string("-") : who),
                               "ms " + std::to_string(ms_since(t0))});
    if (conflicts)
      event(s_, "workdir-sync-conflict", {std::to_string(conflicts) + " shard(s) changed "
                                          "differently by several ranks; lowest rank written"});
    return dirty;
  }

  void release() {
    for (int i = 0; i < n_; ++i) {
      if (s_.host) {
        if (image_[i]) munmap(image_[i], s_.total);
        unlink(shm_path(i).c_str());
      } else if (image_[i]) {
        (void)hipSetDevice(s_.devices[i]);
        (void)hipFree(image_[i]);
      }
      image_[i] = nullptr;
      tpi_loader_destroy(loaders_[i]);
      loaders_[i] = nullptr;
    }
    for (tpi_comm* c : comms_) tpi_comm_destroy(c);
    comms_.clear();
  }

 private:
  Spec s_;
  int n_;
  std::vector<void*> image_;
  std::vector<tpi_loader*> loaders_;
  std::vector<tpi_comm*> comms_;
  std::vector<uint64_t> base_;                 // digests of the staged image (every copy)
  std::vector<std::vector<uint64_t>> bases_;   // per rank: digests of its copy as last synced
  double alloc_ms_ = 0, load_ms_ = 0, read_ms_ = 0, fanout_ms_ = 0, comm_ms_ = 0,
         verify_ms_ = 0;
  bool verified_ = false;

  std::string shm_path(int i) const {
    return s_.shm_prefix + "-" + std::to_string(getpid()) + "-" + std::to_string(i);
  }

  void allocate() {
    image_.assign(n_, nullptr);
    loaders_.assign(n_, nullptr);
    for (int i = 0; i < n_; ++i) {
      if (s_.host) {
        int fd = open(shm_path(i).c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)s_.total)) die("shm image: " + std::string(strerror(errno)));
        void* p = mmap(nullptr, s_.total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) die("mmap image: " + std::string(strerror(errno)));
        image_[i] = p;
      } else {
        hip_check(hipSetDevice(s_.devices[i]), "hipSetDevice");
        hip_check(hipMalloc(&image_[i], std::max<uint64_t>(s_.total, 4096)), "hipMalloc(image)");
      }
      loaders_[i] = tpi_loader_create(s_.host ? -1 : s_.devices[i], s_.chunk, s_.nbuf, s_.threads,
                                      s_.numa[i]);
      if (!loaders_[i]) die(std::string("loader: ") + tpi_last_error());
    }
  }

  // Which image bytes GPU i reads from the host.
  std::pair<uint64_t, uint64_t> load_range(int i) const {
    if (s_.method == "sharded") {
      const uint64_t shard = s_.total / n_;
      return {i * shard, (i + 1) * shard};
    }
    if (s_.method == "broadcast") return {0, i == 0 ? s_.total : 0};
    return {0, s_.total};
  }

  void load() {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    std::vector<std::string> errs(n_);
    std::vector<double> read(n_, 0);
    for (int i = 0; i < n_; ++i) {
      th.emplace_back([&, i] {
        auto r = load_range(i);
        if (r.first >= r.second) return;
        tpi_stats st = {};
        if (tpi_loader_load(loaders_[i], s_.files.data(), s_.files.size(), r.first, r.second,
                            image_[i], &st))
          errs[i] = tpi_last_error();
        read[i] = st.pack_ms;
      });
    }
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (!e.empty()) die("load: " + e);
    load_ms_ = ms_since(t0);
    read_ms_ = *std::max_element(read.begin(), read.end());
  }

  void fanout() {
    if (n_ == 1 || s_.method == "independent") return;
    const uint64_t shard = s_.total / n_;
    if (s_.host) {  // the same schedule with memcpy: shard j of image j -> every image
      auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> th;
      for (int i = 0; i < n_; ++i)
        th.emplace_back([&, i] {
          for (int j = 0; j < n_; ++j) {
            if (s_.method == "sharded" && j != i)
              memcpy((uint8_t*)image_[i] + j * shard, (uint8_t*)image_[j] + j * shard, shard);
          }
          if (s_.method == "broadcast" && i) memcpy(image_[i], image_[0], s_.total);
        });
      for (auto& t : th) t.join();
      fanout_ms_ = ms_since(t0);
      return;
    }
    auto t0 = std::chrono::steady_clock::now();
    comms_.assign(n_, nullptr);
    check(tpi_comm_init_all(n_, s_.devices.data(), comms_.data()), "task communicator");
    comm_ms_ = ms_since(t0);
    t0 = std::chrono::steady_clock::now();
    if (s_.method == "sharded")
      check(tpi_comm_allgather_inplace(comms_.data(), n_, image_.data(), shard, 1), "all-gather");
    else
      check(tpi_comm_broadcast(comms_.data(), n_, image_.data(), s_.total, 0, 1), "broadcast");
    fanout_ms_ = ms_since(t0);
  }

  std::vector<uint64_t> digests(int i) {
    const uint64_t n = (s_.total + s_.shard_bytes - 1) / s_.shard_bytes;
    std::vector<uint64_t> out(n, 0);
    if (n == 0) return out;
    if (s_.host) {
      std::vector<std::thread> th;
      const unsigned nt = std::max(1, s_.threads);
      for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
          for (uint64_t k = t; k < n; k += nt) {
            const uint64_t lo = k * s_.shard_bytes, len = std::min(s_.shard_bytes, s_.total - lo);
            out[k] = tpi_shard_hash_host((const uint8_t*)image_[i] + lo, len, 0);
          }
        });
      for (auto& t : th) t.join();
      return out;
    }
    hip_check(hipSetDevice(s_.devices[i]), "hipSetDevice");
    uint64_t* d = nullptr;
    hip_check(hipMalloc(&d, n * sizeof(uint64_t)), "hipMalloc(digests)");
    check(tpi_shard_hash(image_[i], s_.total, s_.shard_bytes, 0, d, 0), "shard hash");
    hip_check(hipMemcpy(out.data(), d, n * sizeof(uint64_t), hipMemcpyDeviceToHost), "digests D2H");
    hip_check(hipFree(d), "hipFree");
    return out;
  }

  // Rank 0's digests are the sync baseline; with `verify` every other copy must match them.
  void verify() {
    auto t0 = std::chrono::steady_clock::now();
    base_ = digests(0);
    verified_ = true;
    for (int i = 1; i < n_ && s_.verify; ++i) verified_ = verified_ && digests(i) == base_;
    verify_ms_ = ms_since(t0);
    if (!verified_) die("fan-out verification failed: GPU copies differ");
    bases_.assign(n_, base_);
  }

  void publish() {
    std::string ranks;
    for (int i = 0; i < n_; ++i) {
      std::string entry;
      if (s_.host) {
        entry = "{\"path\": " + quote(shm_path(i)) + "}";
      } else {
        uint8_t h[TPI_IPC_HANDLE_BYTES];
        hip_check(hipSetDevice(s_.devices[i]), "hipSetDevice");
        check(tpi_ipc_handle(image_[i], h), "IPC handle");
        entry = "{\"device\": " + std::to_string(s_.devices[i]) + ", \"ipc\": " +
                quote(hex(h, sizeof(h))) + "}";
      }
      ranks += (i ? ", " : "") + entry;
    }
    std::string files;
    for (size_t k = 0; k < s_.files.size(); ++k)
      files += (k ? ", " : "") + std::string("[") + quote(s_.rel[k]) + ", " +
               std::to_string(s_.files[k].offset) + ", " + std::to_string(s_.files[k].size) + "]";
    const double gb = s_.total / 1e9;
    auto rate = [&](double ms) { return ms > 0 ? gb / (ms / 1e3) : 0.0; };
    const std::string stats =
        "{\"bytes\": " + std::to_string(s_.total) + ", \"ranks\": " + std::to_string(n_) +
        ", \"alloc_ms\": " + std::to_string(alloc_ms_) + ", \"load_ms\": " +
        std::to_string(load_ms_) + ", \"read_ms\": " + std::to_string(read_ms_) +
        ", \"comm_init_ms\": " + std::to_string(comm_ms_) + ", \"fanout_ms\": " +
        std::to_string(fanout_ms_) + ", \"verify_ms\": " + std::to_string(verify_ms_) +
        ", \"load_GBps\": " + std::to_string(rate(load_ms_)) + ", \"staged_GBps\": " +
        std::to_string(rate(load_ms_ + fanout_ms_)) + ", \"verified\": " +
        (verified_ ? "true" : "false") + "}";
    const std::string manifest =
        "{\"version\": 1, \"pid\": " + std::to_string(getpid()) + ", \"root\": " +
        quote(s_.root) + ", \"method\": " + quote(s_.method) + ", \"host\": " +
        (s_.host ? "true" : "false") + ", \"total\": " + std::to_string(s_.total) +
        ", \"shard_bytes\": " + std::to_string(s_.shard_bytes) + ", \"ranks\": [" + ranks +
        "], \"files\": [" + files + "], \"stats\": " + stats + "}\n";
    if (!atomic_write(s_.manifest, manifest)) die("cannot write " + s_.manifest);
    event(s_, "staged", {"method " + s_.method, "ranks " + std::to_string(n_),
                         "bytes " + std::to_string(s_.total),
                         "load_ms " + std::to_string(load_ms_),
                         "fanout_ms " + std::to_string(fanout_ms_),
                         "GBps " + std::to_string(rate(load_ms_ + fanout_ms_))});
    printf("staged %s\n", stats.c_str());
    fflush(stdout);
  }
};

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: tpi-stager <stage.json>\n");
    return 2;
  }
  sigset_t mask;
  sigemptyset(&mask);
  for (int sig : {SIGTERM, SIGINT, SIGHUP, SIGUSR1}) sigaddset(&mask, sig);
  sigprocmask(SIG_BLOCK, &mask, nullptr);
  Spec spec = load_spec(argv[1]);
  const double interval = spec.sync_interval;
  const bool sync_on = spec.writeback && interval > 0;
  Stager stager(std::move(spec));
  stager.stage();
  // Hold the images until the supervisor ends the task; sync on the cadence / on demand.
  while (true) {
    struct timespec ts = {1000000, 0};
    if (sync_on) {
      ts.tv_sec = (time_t)interval;
      ts.tv_nsec = (long)((interval - (double)ts.tv_sec) * 1e9);
    }
    int sig = sigtimedwait(&mask, nullptr, &ts);
    if (sig < 0 && errno == EINTR) continue;
    if (sig < 0) {  // cadence tick
      if (sync_on) stager.sync("interval");
      continue;
    }
    if (sig == SIGUSR1) {
      stager.sync("request");
      continue;
    }
    if (sync_on) stager.sync("final");
    break;
  }
  stager.release();
  return 0;
}
