// Host memory of the engine (engine_internal.h): NUMA-local file-backed mappings, their
// registration (whole, or window by window with a tpi_pinner), the engine's host region
// and progress words, and the plain H2D / D2H entry points.
#include "engine_internal.h"

using namespace tpi_engine_detail;

extern "C" {

// ---- host memory ---------------------------------------------------------------------------

void* tpi_host_map(const char* path, uint64_t bytes, int numa_node, int populate) {
  int fd = -1;
  int flags = MAP_PRIVATE | MAP_ANONYMOUS;
  if (path && *path) {
    fd = open(path, O_RDWR | O_CREAT, 0600);
    if (fd < 0) {
      fail(std::string("open ") + path + ": " + strerror(errno));
      return nullptr;
    }
    struct stat st;
    if (fstat(fd, &st) == 0 && (uint64_t)st.st_size < bytes && ftruncate(fd, bytes) != 0) {
      fail(std::string("ftruncate: ") + strerror(errno));
      close(fd);
      return nullptr;
    }
    flags = MAP_SHARED;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, flags, fd, 0);
  if (fd >= 0) close(fd);
  if (p == MAP_FAILED) {
    fail(std::string("mmap: ") + strerror(errno));
    return nullptr;
  }
  madvise(p, bytes, MADV_HUGEPAGE);
  if (numa_node >= 0 && numa_node < 1024) {
    unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
    mask[numa_node / (8 * sizeof(unsigned long))] |= 1ul << (numa_node % (8 * sizeof(unsigned long)));
    // MPOL_PREFERRED = 1: fall back to other nodes instead of failing under pressure.
    syscall(SYS_mbind, p, bytes, 1, mask, 1024, 0);
  }
  if (populate) {
    // Parallel first touch: page faults dominate, one thread per ~1 GiB up to 16.
    const uint64_t page = 4096;
    unsigned nth = (unsigned)std::min<uint64_t>(16, std::max<uint64_t>(1, bytes >> 30));
    std::vector<std::thread> th;
    const uint64_t per = ((bytes / nth) + page - 1) / page * page;
    for (unsigned i = 0; i < nth; ++i) {
      th.emplace_back([=] {
        uint64_t b = (uint64_t)i * per, e = std::min(bytes, b + per);
        volatile uint8_t* q = (volatile uint8_t*)p;
        for (uint64_t o = b; o < e; o += page) q[o] = q[o];
      });
    }
    for (auto& t : th) t.join();
  }
  return p;
}

int tpi_host_unmap(void* ptr, uint64_t bytes) {
  if (munmap(ptr, bytes)) return fail(std::string("munmap: ") + strerror(errno));
  return 0;
}

int tpi_host_register(void* ptr, uint64_t bytes) {
  HIP_OK(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  return 0;
}

int tpi_host_register_ro(void* ptr, uint64_t bytes) {
  HIP_OK(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterReadOnly));
  return 0;
}

int tpi_h2d_async(void* dev_dst, const void* host_src, uint64_t bytes, uint64_t stream) {
  HIP_OK(hipMemcpyAsync(dev_dst, host_src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return 0;
}

tpi_pinner* tpi_host_pin_start(void* base, uint64_t bytes, uint64_t window, int threads) {
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) device = 0;
  auto* p = new tpi_pinner();
  p->base = (uint8_t*)base;
  p->bytes = bytes;
  p->window = std::max<uint64_t>(2ull << 20, window / (2ull << 20) * (2ull << 20));
  p->threads = std::max(1, threads);
  p->device = device;
  p->toucher = std::thread([p] {
    constexpr uint64_t page = 4096;
    for (uint64_t w = 0; w < p->bytes && !p->stop.load(); w += p->window) {
      const uint64_t end = std::min(p->bytes, w + p->window);
      const uint64_t per = ((end - w) / p->threads + page - 1) / page * page;
      std::vector<std::thread> pool;
      for (int t = 0; t < p->threads; ++t)
        pool.emplace_back([p, w, end, per, t] {
          const uint64_t b = w + (uint64_t)t * per, e = std::min(end, b + per);
          volatile const uint8_t* q = p->base;
          uint8_t sink = 0;
          for (uint64_t o = b; o < e; o += page) sink ^= q[o];  // read fault: no data change
          (void)sink;
        });
      for (auto& t : pool) t.join();
      p->touched.store(end, std::memory_order_release);
    }
  });
  p->registrar = std::thread([p] {
    (void)hipSetDevice(p->device);
    for (uint64_t w = 0; w < p->bytes && !p->stop.load(); w += p->window) {
      const uint64_t end = std::min(p->bytes, w + p->window);
      while ((p->touched.load(std::memory_order_acquire) < end ||
              p->held.load(std::memory_order_acquire)) && !p->stop.load())
        std::this_thread::sleep_for(std::chrono::microseconds(100));
      if (p->stop.load()) break;
      hipError_t err = hipHostRegister(p->base + w, end - w,
                                       hipHostRegisterMapped | hipHostRegisterPortable);
      if (err != hipSuccess) {
        p->error = std::string("hipHostRegister(window) : ") + hipGetErrorString(err);
        p->failed.store(true);
        return;
      }
      p->registered.push_back(p->base + w);
      p->ready.store(end, std::memory_order_release);
    }
  });
  return p;
}

uint64_t tpi_host_pin_ready(const tpi_pinner* p) { return p->ready.load(); }

int tpi_host_pin_hold(tpi_pinner* p, int hold) {
  p->held.store(hold != 0, std::memory_order_release);
  return 0;
}
uint64_t tpi_host_pin_window(const tpi_pinner* p) { return p->window; }

// Wait for the whole region (0) or report the pinning error (-1).
int tpi_host_pin_wait(tpi_pinner* p) {
  p->held.store(false, std::memory_order_release);
  if (p->toucher.joinable()) p->toucher.join();
  if (p->registrar.joinable()) p->registrar.join();
  if (p->failed.load()) return fail(p->error);
  return 0;
}

// Stop (if still running), unregister every pinned window, free the pinner.
int tpi_host_pin_release(tpi_pinner* p) {
  if (!p) return 0;
  p->stop.store(true);
  if (p->toucher.joinable()) p->toucher.join();
  if (p->registrar.joinable()) p->registrar.join();
  for (uint8_t* w : p->registered) (void)hipHostUnregister(w);
  delete p;
  return 0;
}

int tpi_engine_set_host_region(tpi_engine* e, void* base, uint64_t bytes, uint64_t window,
                               tpi_pinner* pinner) {
  std::lock_guard<std::mutex> lk(e->mu);
  e->hbase = (const uint8_t*)base;
  e->hbytes = bytes;
  e->hwin = window;
  e->pinner = pinner;
  return 0;
}

// Allocate now what the pipelines would allocate on first use (segment descriptors, tile
// CRCs, the codec's decode buffers): a successor that restores while its predecessor frees
// HBM must not meet a hipMalloc that waits for the driver to clear that memory.
int tpi_engine_alloc_staging(tpi_engine* e) {
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_OK(hipSetDevice(e->device));
  return ensure_staging(e);
}

int tpi_engine_reserve(tpi_engine* e, int nsegs, uint64_t ntiles, int codec) {
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_OK(hipSetDevice(e->device));
  if (ensure_staging(e)) return -1;  // a restore through the host needs the ring
  if ((size_t)nsegs > e->seg_cap) {
    if (e->d_segs) HIP_OK(hipFree(e->d_segs));
    e->d_segs = nullptr;
    e->seg_cap = 0;
    HIP_OK(hipMalloc(&e->d_segs, (size_t)nsegs * sizeof(tpi_seg)));
    e->seg_cap = nsegs;
  }
  if (ntiles > e->crc_cap) {
    if (e->d_crcs) HIP_OK(hipFree(e->d_crcs));
    e->d_crcs = nullptr;
    e->crc_cap = 0;
    HIP_OK(hipMalloc(&e->d_crcs, ntiles * sizeof(uint32_t)));
    e->crc_cap = ntiles;
  }
  // the HBM hand-off's buffers as well: a successor's first copy then allocates nothing
  if (ntiles > e->digest_cap) {
    if (e->d_digest) HIP_OK(hipFree(e->d_digest));
    e->d_digest = nullptr;
    e->digest_cap = 0;
    HIP_OK(hipMalloc(&e->d_digest, ntiles * sizeof(uint64_t)));
    e->digest_cap = ntiles;
  }
  if ((size_t)nsegs > e->src_cap) {
    if (e->d_src) HIP_OK(hipFree(e->d_src));
    e->d_src = nullptr;
    e->src_cap = 0;
    HIP_OK(hipMalloc(&e->d_src, (size_t)nsegs * sizeof(tpi_seg)));
    e->src_cap = nsegs;
  }
  if (codec && prepare_codec(e, ntiles)) return -1;
  return 0;
}

int tpi_engine_set_h2d_sdma(tpi_engine* e, int on) {
  std::lock_guard<std::mutex> lk(e->mu);
  if (!on) {
    tpi_sdma_close(e->sdma_in);
    e->sdma_in = nullptr;
    return 0;
  }
  if (!e->sdma_in) e->sdma_in = tpi_sdma_open_h2d(e->device, e->nbuf);
  return e->sdma_in ? (int)(31 - __builtin_clz(tpi_sdma_engine(e->sdma_in))) : -1;
}

int tpi_engine_set_progress(tpi_engine* e, uint64_t* words) {
  std::lock_guard<std::mutex> lk(e->mu);
  e->progress = words;
  return 0;
}

int tpi_host_unregister(void* ptr) {
  HIP_OK(hipHostUnregister(ptr));
  return 0;
}

int tpi_h2d(tpi_engine* e, void* dev_dst, const void* host_src, uint64_t bytes) {
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(region_copy(e, dev_dst, host_src, bytes, hipMemcpyHostToDevice, e->copy));
  HIP_OK(hipStreamSynchronize(e->copy));
  return 0;
}

int tpi_d2h(tpi_engine* e, void* host_dst, const void* dev_src, uint64_t bytes) {
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_OK(hipSetDevice(e->device));
  if (e->sdma) {
    if (sdma_region_d2h(e, e->nbuf, host_dst, dev_src, bytes)) return -1;
    return tpi_sdma_wait(e->sdma, e->nbuf);
  }
  HIP_OK(region_copy(e, host_dst, dev_src, bytes, hipMemcpyDeviceToHost, e->copy));
  HIP_OK(hipStreamSynchronize(e->copy));
  return 0;
}

}  // extern "C"
