// Workdir staging: host files -> HBM image, HBM image -> host files,
// HIP IPC export/import of the image, and the per-task RCCL communicator.
//
// The reference restores a task's workdir on every machine with an independent
// `rclone copy $RCLONE_REMOTE/data /opt/task/directory` (machine-script.sh.tpl:89), i.e. every
// replica pulls the whole tree over its own network link.  Here a workdir becomes one flat
// image (files at 4 KiB-aligned offsets, gaps zero) resident in HBM on every GPU of the task:
//
//   loader   per GPU: a NUMA-local pinned ring of `nbuf` chunks; `threads` workers pread the
//            files' pieces of chunk k+1 from the page cache while chunk k is in flight H2D on the
//            loader's copy stream -- the H2D link never waits for the disk/page-cache reads.
//   comm     the image is split into N equal shards; GPU i loads only shard i over its own
//            PCIe link, then one in-place RCCL all-gather over xGMI completes every copy: host
//            bytes cross PCIe once in total (not N times), and the all-gather uses every
//            point-to-point xGMI link of the 8-GPU mesh instead of one broadcast ring.
//   ipc      the image's HIP IPC handle, so rank processes map it zero-copy (runtime/stage.py).
//   store    the inverse of the loader for the periodic write-back of dirty shards
//            (machine-script.sh.tpl:118-124: re-sync the workdir every 10 s).
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "internal.h"
#include "tpi_hip.h"

namespace {

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// CPUs of NUMA node `node` (sysfs cpulist "0-63,128-191"); false if unknown.
bool node_cpus(int node, cpu_set_t* set) {
  if (node < 0) return false;
  FILE* f = fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
  if (!f) return false;
  char buf[4096] = {0};
  const bool ok = fgets(buf, sizeof(buf), f) != nullptr;
  fclose(f);
  if (!ok) return false;
  CPU_ZERO(set);
  int count = 0;
  for (char* p = buf; *p && *p != '\n';) {
    char* end = nullptr;
    long lo = strtol(p, &end, 10), hi = lo;
    if (end == p) break;
    if (*end == '-') hi = strtol(end + 1, &end, 10);
    for (long c = lo; c <= hi && c < CPU_SETSIZE; ++c, ++count) CPU_SET((int)c, set);
    p = *end == ',' ? end + 1 : end;
  }
  return count > 0;
}

// Fork-join pool: run(fn) calls fn(0..n-1) once each (fn(0) on the caller) and returns when
// all are done.  Workers sleep on a condition variable between jobs.  With `cpus`, the
// workers run on those CPUs (the NUMA node of the pinned ring they fill), so the page-cache
// copies write the ring from its own socket instead of across the inter-socket link.
class Pool {
 public:
  explicit Pool(int n, const cpu_set_t* cpus = nullptr) : n_(std::max(1, n)) {
    for (int i = 1; i < n_; ++i) {
      workers_.emplace_back([this, i] { loop(i); });
      if (cpus) pthread_setaffinity_np(workers_.back().native_handle(), sizeof(*cpus), cpus);
    }
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return n_; }
  void run(const std::function<void(int)>& fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &fn;
      pending_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(int i) {
    uint64_t seen = 0;
    while (true) {
      const std::function<void(int)>* job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (quit_) return;
        job = job_;
      }
      (*job)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }
  int n_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool quit_ = false;
};

// First file whose bytes end after `pos` (files sorted by offset).
uint64_t first_file(const tpi_file* files, uint64_t n, uint64_t pos) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (files[mid].offset + files[mid].size <= pos) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Fill buf with image bytes [a, b): file pieces read with pread, gaps zeroed.
// Returns an error text ("" = ok).
std::string read_range(const tpi_file* files, uint64_t n, uint64_t a, uint64_t b, uint8_t* buf) {
  uint64_t cur = a;
  for (uint64_t i = first_file(files, n, a); i < n && files[i].offset < b; ++i) {
    const uint64_t s = std::max(a, files[i].offset);
    const uint64_t e = std::min(b, files[i].offset + files[i].size);
    if (s >= e) continue;
    if (s > cur) memset(buf + (cur - a), 0, s - cur);
    int fd = open(files[i].path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return std::string("open ") + files[i].path + ": " + strerror(errno);
    uint64_t done = 0;
    while (done < e - s) {
      ssize_t r = pread(fd, buf + (s - a) + done, e - s - done, (off_t)(s - files[i].offset + done));
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) {
        close(fd);
        return std::string("read ") + files[i].path + ": " + (r < 0 ? strerror(errno) : "file shrank");
      }
      done += (uint64_t)r;
    }
    close(fd);
    cur = e;
  }
  if (cur < b) memset(buf + (cur - a), 0, b - cur);
  return "";
}

// Write image bytes [a, b) (held in buf) back into the files they belong to.
std::string write_range(const tpi_file* files, uint64_t n, uint64_t a, uint64_t b,
                        const uint8_t* buf) {
  for (uint64_t i = first_file(files, n, a); i < n && files[i].offset < b; ++i) {
    const uint64_t s = std::max(a, files[i].offset);
    const uint64_t e = std::min(b, files[i].offset + files[i].size);
    if (s >= e) continue;
    int fd = open(files[i].path, O_WRONLY | O_CLOEXEC);
    if (fd < 0) return std::string("open ") + files[i].path + ": " + strerror(errno);
    uint64_t done = 0;
    while (done < e - s) {
      ssize_t w = pwrite(fd, buf + (s - a) + done, e - s - done, (off_t)(s - files[i].offset + done));
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) {
        close(fd);
        return std::string("write ") + files[i].path + ": " + strerror(errno);
      }
      done += (uint64_t)w;
    }
    close(fd);
  }
  return "";
}

// Split [a, b) into `parts` page-aligned slices and run fn(slice_lo, slice_hi) on the pool.
std::string parallel_ranges(Pool& pool, uint64_t a, uint64_t b,
                            const std::function<std::string(uint64_t, uint64_t)>& fn) {
  const int parts = pool.size();
  const uint64_t per = ((b - a + parts - 1) / parts + 4095) / 4096 * 4096;
  std::vector<std::string> errs(parts);
  pool.run([&](int i) {
    const uint64_t lo = a + (uint64_t)i * per, hi = std::min(b, lo + per);
    if (lo < hi) errs[i] = fn(lo, hi);
  });
  for (auto& e : errs)
    if (!e.empty()) return e;
  return "";
}

}  // namespace

struct tpi_loader {
  int device = -1;  // -1: the image is host memory
  uint64_t chunk = 0;
  int nbuf = 0;
  Pool* pool = nullptr;
  std::vector<uint8_t*> ring;  // pinned, NUMA-local
  std::vector<hipEvent_t> ev;
  hipStream_t stream = nullptr;
  uint64_t ring_bytes = 0;
};

extern "C" {

tpi_loader* tpi_loader_create(int device, uint64_t chunk_bytes, int nbuf, int threads,
                              int numa_node) {
  auto* L = new tpi_loader();
  L->device = device;
  L->chunk = std::max<uint64_t>(4096, chunk_bytes / 4096 * 4096);
  L->nbuf = std::max(2, nbuf);
  cpu_set_t cpus;
  const char* pin = getenv("TPI_STAGE_PIN_THREADS");
  const bool bind = !(pin && pin[0] == '0') && node_cpus(numa_node, &cpus);
  L->pool = new Pool(std::max(1, threads), bind ? &cpus : nullptr);
  if (device >= 0) {
    auto bail = [&](const std::string& what) -> tpi_loader* {
      tpi_fail(what);
      tpi_loader_destroy(L);
      return nullptr;
    };
    hipError_t err;
    if ((err = hipSetDevice(device)) != hipSuccess)
      return bail(std::string("hipSetDevice: ") + hipGetErrorString(err));
    if ((err = hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking)) != hipSuccess)
      return bail(std::string("hipStreamCreate: ") + hipGetErrorString(err));
    L->ring_bytes = L->chunk * L->nbuf;
    void* ring = tpi_host_map(nullptr, L->ring_bytes, numa_node, 1);
    if (!ring) return bail("pinned ring: host map failed");
    if (tpi_host_register(ring, L->ring_bytes)) {
      tpi_host_unmap(ring, L->ring_bytes);
      return bail("pinned ring: hipHostRegister failed");
    }
    for (int i = 0; i < L->nbuf; ++i) {
      L->ring.push_back((uint8_t*)ring + (uint64_t)i * L->chunk);
      hipEvent_t e = nullptr;
      if ((err = hipEventCreateWithFlags(&e, hipEventDisableTiming)) != hipSuccess)
        return bail(std::string("hipEventCreate: ") + hipGetErrorString(err));
      L->ev.push_back(e);
    }
  }
  return L;
}

void tpi_loader_destroy(tpi_loader* L) {
  if (!L) return;
  if (L->device >= 0) {
    (void)hipSetDevice(L->device);
    if (L->stream) (void)hipStreamSynchronize(L->stream);
    for (hipEvent_t e : L->ev)
      if (e) (void)hipEventDestroy(e);
    if (!L->ring.empty()) {
      (void)hipHostUnregister(L->ring[0]);
      tpi_host_unmap(L->ring[0], L->ring_bytes);
    }
    if (L->stream) (void)hipStreamDestroy(L->stream);
  }
  delete L->pool;
  delete L;
}

int tpi_loader_load(tpi_loader* L, const tpi_file* files, uint64_t nfiles, uint64_t lo,
                    uint64_t hi, void* dst, tpi_stats* stats) {
  roctxRangePushA("tpi_loader_load");
  auto t0 = std::chrono::steady_clock::now();
  double read_ms = 0;
  uint64_t chunks = 0;
  int rc = 0;
  if (L->device < 0) {  // host image: read straight into it
    auto r0 = std::chrono::steady_clock::now();
    std::string err = parallel_ranges(*L->pool, lo, hi, [&](uint64_t a, uint64_t b) {
      return read_range(files, nfiles, a, b, (uint8_t*)dst + a);
    });
    read_ms = ms_since(r0);
    chunks = 1;
    if (!err.empty()) rc = tpi_fail(err);
  } else {
    rc = [&]() -> int {
      TPI_HIP(hipSetDevice(L->device));
      for (uint64_t a = lo, k = 0; a < hi; a += L->chunk, ++k) {
        const int slot = (int)(k % L->nbuf);
        const uint64_t b = std::min(hi, a + L->chunk);
        if (k >= (uint64_t)L->nbuf) TPI_HIP(hipEventSynchronize(L->ev[slot]));
        auto r0 = std::chrono::steady_clock::now();
        uint8_t* host = L->ring[slot];
        std::string err = parallel_ranges(*L->pool, a, b, [&](uint64_t x, uint64_t y) {
          return read_range(files, nfiles, x, y, host + (x - a));
        });
        read_ms += ms_since(r0);
        if (!err.empty()) return tpi_fail(err);
        TPI_HIP(hipMemcpyAsync((uint8_t*)dst + a, host, b - a, hipMemcpyHostToDevice, L->stream));
        TPI_HIP(hipEventRecord(L->ev[slot], L->stream));
        chunks = k + 1;
      }
      TPI_HIP(hipStreamSynchronize(L->stream));
      return 0;
    }();
  }
  if (stats) {
    stats->copy_ms = ms_since(t0);
    stats->pack_ms = read_ms;  // host time spent reading files (overlaps the copies)
    stats->bytes = hi - lo;
    stats->chunks = chunks;
  }
  roctxRangePop();
  return rc;
}

// Write-back: image ranges -> files.  Device images go through the pinned ring: the D2H of
// the next nbuf-1 chunks is in flight on the copy stream while the pool writes the current
// one, so the PCIe leg and the file writes overlap (the mirror of tpi_loader_load).
int tpi_loader_store(tpi_loader* L, const tpi_file* files, uint64_t nfiles,
                     const uint64_t* ranges, uint64_t nranges, const void* src,
                     tpi_stats* stats) {
  roctxRangePushA("tpi_loader_store");
  auto t0 = std::chrono::steady_clock::now();
  uint64_t bytes = 0, chunks = 0;
  struct Piece {
    uint64_t a, b;
  };
  std::vector<Piece> pieces;  // every chunk of every range, in order
  for (uint64_t r = 0; r < nranges; ++r)
    for (uint64_t a = ranges[2 * r]; a < ranges[2 * r + 1]; a += L->chunk)
      pieces.push_back({a, std::min(ranges[2 * r + 1], a + L->chunk)});
  int rc = [&]() -> int {
    auto write = [&](const Piece& p, const uint8_t* host) -> int {
      std::string err = parallel_ranges(*L->pool, p.a, p.b, [&](uint64_t x, uint64_t y) {
        return write_range(files, nfiles, x, y, host + (x - p.a));
      });
      if (!err.empty()) return tpi_fail(err);
      bytes += p.b - p.a;
      ++chunks;
      return 0;
    };
    if (L->device < 0) {
      for (auto& p : pieces)
        if (write(p, (const uint8_t*)src + p.a)) return -1;
      return 0;
    }
    TPI_HIP(hipSetDevice(L->device));
    const size_t depth = (size_t)L->nbuf;
    size_t issued = 0;
    auto issue = [&](size_t k) -> int {
      const int slot = (int)(k % depth);
      TPI_HIP(hipMemcpyAsync(L->ring[slot], (const uint8_t*)src + pieces[k].a,
                             pieces[k].b - pieces[k].a, hipMemcpyDeviceToHost, L->stream));
      TPI_HIP(hipEventRecord(L->ev[slot], L->stream));
      return 0;
    };
    for (size_t k = 0; k < pieces.size(); ++k) {
      // keep up to nbuf - 1 copies ahead of the chunk being written (its slot stays busy)
      while (issued < pieces.size() && issued < k + depth - 1 + (depth == 1)) {
        if (issue(issued)) return -1;
        ++issued;
      }
      const int slot = (int)(k % depth);
      TPI_HIP(hipEventSynchronize(L->ev[slot]));
      if (write(pieces[k], L->ring[slot])) {
        (void)hipStreamSynchronize(L->stream);  // no copy may land in a ring we give up
        return -1;
      }
    }
    return 0;
  }();
  if (stats) {
    stats->copy_ms = ms_since(t0);
    stats->pack_ms = 0;
    stats->bytes = bytes;
    stats->chunks = chunks;
  }
  roctxRangePop();
  return rc;
}

// ---- HIP IPC -------------------------------------------------------------------------------

int tpi_ipc_handle(void* dev_ptr, uint8_t* out) {
  hipIpcMemHandle_t h;
  TPI_HIP(hipIpcGetMemHandle(&h, dev_ptr));
  memcpy(out, &h, sizeof(h));
  return 0;
}

int tpi_ipc_open(const uint8_t* handle, int device, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  TPI_HIP(hipSetDevice(device));
  TPI_HIP(hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess));
  return 0;
}

int tpi_ipc_close(void* dev_ptr) {
  TPI_HIP(hipIpcCloseMemHandle(dev_ptr));
  return 0;
}

// One plain hipMalloc outside PyTorch's caching allocator (whose cached segments can be split
// into a request, leaving it inside a larger allocation): the hand-off relocates tensors of
// allocations HIP IPC cannot open into such blocks (checkpoint/checkpointer.py).
int tpi_dev_alloc(uint64_t bytes, void** out) {
  TPI_HIP(hipMalloc(out, (size_t)bytes));
  return 0;
}

int tpi_dev_free(void* ptr) {
  TPI_HIP(hipFree(ptr));
  return 0;
}

// Device-to-device copy on `stream` (0: the null stream), synchronous.
int tpi_d2d(void* dst, const void* src, uint64_t bytes, uint64_t stream) {
  TPI_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  TPI_HIP(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

}  // extern "C"

// ---- task communicator (RCCL) ----------------------------------------------------------------

struct tpi_comm {
  ncclComm_t comm = nullptr;
  int device = 0, rank = 0, nranks = 1;
  hipStream_t stream = nullptr;
};

namespace {

#define TPI_NCCL(expr)                                                                   \
  do {                                                                                   \
    ncclResult_t r_ = (expr);                                                            \
    if (r_ != ncclSuccess) return tpi_fail(std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

int comm_stream(tpi_comm* c) {
  TPI_HIP(hipSetDevice(c->device));
  TPI_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  return 0;
}

// Collectives of several ranks are enqueued in one NCCL group.  Whatever fails -- an enqueue
// or the group end -- the group is ended before returning: a thread left inside
// ncclGroupStart() would silently fold every later NCCL call into that unfinished group.
// TPI_NCCL_FAIL_AT=<i> (fault injection, tests) fails the i-th enqueue without calling NCCL.
thread_local int g_groups_open = 0;  // NCCL group depth is per thread

template <class Enqueue>
int grouped(const char* what, int n, Enqueue&& enqueue) {
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return tpi_fail(std::string("ncclGroupStart: ") + ncclGetErrorString(r));
  ++g_groups_open;
  int fail_at = -1;
  if (const char* f = getenv("TPI_NCCL_FAIL_AT")) fail_at = atoi(f);
  ncclResult_t first = ncclSuccess;
  int at = -1;
  for (int i = 0; i < n && first == ncclSuccess; ++i) {
    const ncclResult_t e = i == fail_at ? ncclInvalidArgument : enqueue(i);
    if (e != ncclSuccess) {
      first = e;
      at = i;
    }
  }
  const ncclResult_t end = ncclGroupEnd();
  --g_groups_open;
  if (first != ncclSuccess)
    return tpi_fail(std::string(what) + " (rank " + std::to_string(at) + "): " +
                    ncclGetErrorString(first) + (end != ncclSuccess ? std::string("; ncclGroupEnd: ") +
                                                     ncclGetErrorString(end) : std::string()));
  if (end != ncclSuccess) return tpi_fail(std::string("ncclGroupEnd: ") + ncclGetErrorString(end));
  return 0;
}

int finish(tpi_comm** comms, int n, int sync) {
  if (!sync) return 0;
  for (int i = 0; i < n; ++i) {
    TPI_HIP(hipSetDevice(comms[i]->device));
    TPI_HIP(hipStreamSynchronize(comms[i]->stream));
  }
  return 0;
}

}  // namespace

extern "C" {

int tpi_comm_unique_id(uint8_t* out) {
  ncclUniqueId id;
  TPI_NCCL(ncclGetUniqueId(&id));
  memcpy(out, &id, sizeof(id));
  return 0;
}

tpi_comm* tpi_comm_init_rank(const uint8_t* id_bytes, int nranks, int rank, int device) {
  auto* c = new tpi_comm();
  c->device = device;
  c->rank = rank;
  c->nranks = nranks;
  ncclUniqueId id;
  memcpy(&id, id_bytes, sizeof(id));
  hipError_t e = hipSetDevice(device);
  ncclResult_t r = e == hipSuccess ? ncclCommInitRank(&c->comm, nranks, id, rank) : ncclSuccess;
  if (e != hipSuccess || r != ncclSuccess || comm_stream(c)) {
    if (e != hipSuccess) tpi_fail(std::string("hipSetDevice: ") + hipGetErrorString(e));
    else if (r != ncclSuccess) tpi_fail(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    tpi_comm_destroy(c);
    return nullptr;
  }
  return c;
}

int tpi_comm_init_all(int ndev, const int* devices, tpi_comm** out) {
  for (int i = 0; i < ndev; ++i) out[i] = nullptr;
  std::vector<ncclComm_t> raw(ndev, nullptr);
  TPI_NCCL(ncclCommInitAll(raw.data(), ndev, devices));
  for (int i = 0; i < ndev; ++i) {
    out[i] = new tpi_comm();
    out[i]->comm = raw[i];
    raw[i] = nullptr;  // owned by out[i] now
    out[i]->device = devices[i];
    out[i]->rank = i;
    out[i]->nranks = ndev;
    if (comm_stream(out[i])) {
      // a partial set is useless (every collective needs all ranks): release all of it
      const std::string why = tpi_last_error();
      for (int j = 0; j < ndev; ++j) {
        tpi_comm_destroy(out[j]);
        out[j] = nullptr;
        if (raw[j]) (void)ncclCommDestroy(raw[j]);
      }
      return tpi_fail("task communicator stream: " + why);
    }
  }
  return 0;
}

void tpi_comm_destroy(tpi_comm* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int tpi_comm_rank(const tpi_comm* c) { return c->rank; }
int tpi_comm_size(const tpi_comm* c) { return c->nranks; }

int tpi_comm_allgather_inplace(tpi_comm** comms, int n, void** bufs, uint64_t shard_bytes,
                               int sync) {
  roctxRangePushA("tpi_comm_allgather");
  int rc = grouped("ncclAllGather", n, [&](int i) {
    uint8_t* b = (uint8_t*)bufs[i];
    return ncclAllGather(b + (uint64_t)comms[i]->rank * shard_bytes, b, shard_bytes, ncclUint8,
                         comms[i]->comm, comms[i]->stream);
  });
  if (rc == 0) rc = finish(comms, n, sync);
  roctxRangePop();
  return rc;
}

int tpi_comm_broadcast(tpi_comm** comms, int n, void** bufs, uint64_t bytes, int root, int sync) {
  roctxRangePushA("tpi_comm_broadcast");
  int rc = grouped("ncclBroadcast", n, [&](int i) {
    return ncclBroadcast(bufs[i], bufs[i], bytes, ncclUint8, root, comms[i]->comm,
                         comms[i]->stream);
  });
  if (rc == 0) rc = finish(comms, n, sync);
  roctxRangePop();
  return rc;
}

int tpi_nccl_groups_open() { return g_groups_open; }

int tpi_comm_sync(tpi_comm** comms, int n) { return finish(comms, n, 1); }

}  // extern "C"
