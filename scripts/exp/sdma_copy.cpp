// Experiment: device -> pinned host copies through the HIP runtime vs straight onto the SDMA
// engines through HSA (hsa_amd_memory_async_copy_on_engine).  hipMemcpyAsync D2H runs as
// __amd_rocclr_copyBuffer blit kernels on this image (rocprofv3 of copy_engines.py); this
// measures what the copy engines themselves reach, one engine and split over several.
//
//   hipcc -O2 -std=c++17 scripts/exp/sdma_copy.cpp -lhsa-runtime64 -o scripts/exp/sdma_copy
//   ./sdma_copy [GiB] [register|thp|hostmalloc]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <sys/mman.h>
#include <vector>

#define HIPCK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)
#define HSACK(x)                                                                 \
  do {                                                                           \
    hsa_status_t s_ = (x);                                                       \
    if (s_ != HSA_STATUS_SUCCESS) {                                              \
      const char* m_ = nullptr;                                                  \
      hsa_status_string(s_, &m_);                                                \
      fprintf(stderr, "%s: %s\n", #x, m_ ? m_ : "?");                            \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

struct Agents {
  uint32_t bdf = 0;
  hsa_agent_t gpu{}, cpu{};
  bool found = false;
};

static hsa_status_t find_gpu(hsa_agent_t a, void* data) {
  Agents* g = (Agents*)data;
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0;
  hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
  if (bdf == g->bdf) {
    g->gpu = a;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NEAREST_CPU, &g->cpu);
    g->found = true;
  }
  return HSA_STATUS_SUCCESS;
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 1.0;
  const std::string kind = argc > 2 ? argv[2] : "register";
  const bool reg = kind != "hostmalloc";
  const bool thp = kind == "thp";  // anonymous mapping with transparent huge pages
  const size_t n = (size_t)(gib * (1ull << 30));
  HIPCK(hipSetDevice(0));
  hipDeviceProp_t p;
  HIPCK(hipGetDeviceProperties(&p, 0));
  Agents ag;
  ag.bdf = (uint32_t)((p.pciBusID << 8) | (p.pciDeviceID << 3));
  HSACK(hsa_init());
  HSACK(hsa_iterate_agents(find_gpu, &ag));
  if (!ag.found) {
    fprintf(stderr, "no HSA agent with BDF 0x%x\n", ag.bdf);
    return 1;
  }
  uint32_t nsdma = 0, nxgmi = 0;
  hsa_agent_get_info(ag.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NUM_SDMA_ENG, &nsdma);
  hsa_agent_get_info(ag.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NUM_SDMA_XGMI_ENG, &nxgmi);
  uint32_t d2h_mask = 0, h2d_mask = 0, d2h_pref = 0, h2d_pref = 0;
  hsa_amd_memory_copy_engine_status(ag.cpu, ag.gpu, &d2h_mask);
  hsa_amd_memory_copy_engine_status(ag.gpu, ag.cpu, &h2d_mask);
  hsa_amd_memory_get_preferred_copy_engine(ag.cpu, ag.gpu, &d2h_pref);
  hsa_amd_memory_get_preferred_copy_engine(ag.gpu, ag.cpu, &h2d_pref);
  printf("bdf 0x%x sdma %u xgmi_sdma %u d2h_mask 0x%x h2d_mask 0x%x d2h_pref 0x%x h2d_pref 0x%x\n",
         ag.bdf, nsdma, nxgmi, d2h_mask, h2d_mask, d2h_pref, h2d_pref);

  void* dev = nullptr;
  HIPCK(hipMalloc(&dev, n));
  HIPCK(hipMemset(dev, 7, n));
  void* host = nullptr;
  if (reg) {
    host = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (thp) madvise(host, n, MADV_HUGEPAGE);
    memset(host, 1, n);
    HIPCK(hipHostRegister(host, n, hipHostRegisterMapped | hipHostRegisterPortable));
  } else {
    HIPCK(hipHostMalloc(&host, n, 0));
    memset(host, 1, n);
  }
  void* hdev = nullptr;
  HIPCK(hipHostGetDevicePointer(&hdev, host, 0));
  printf("host %p device view %p (%s)\n", host, hdev, host == hdev ? "same" : "differs");
  hipStream_t s;
  HIPCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int reps = 6;

  for (int dir = 0; dir < 2; ++dir) {  // 0 = D2H, 1 = H2D
    const char* dn = dir == 0 ? "d2h" : "h2d";
    void* dst = dir == 0 ? hdev : dev;
    void* src = dir == 0 ? dev : hdev;
    hipMemcpyKind k = dir == 0 ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice;
    HIPCK(hipMemcpyAsync(dst, src, n, k, s));
    HIPCK(hipStreamSynchronize(s));
    double t0 = now();
    for (int r = 0; r < reps; ++r) HIPCK(hipMemcpyAsync(dst, src, n, k, s));
    HIPCK(hipStreamSynchronize(s));
    printf("%s hipMemcpyAsync        %.1f GB/s\n", dn, reps * n / (now() - t0) / 1e9);

    hsa_agent_t da = dir == 0 ? ag.cpu : ag.gpu, sa = dir == 0 ? ag.gpu : ag.cpu;
    uint32_t mask = dir == 0 ? d2h_mask : h2d_mask;
    std::vector<uint32_t> engines;
    for (int b = 0; b < 16; ++b)
      if (mask & (1u << b)) engines.push_back(1u << b);
    hsa_signal_t sig;
    HSACK(hsa_signal_create(1, 0, nullptr, &sig));
    // runtime-chosen engine
    {
      double t = 0;
      for (int r = -1; r < reps; ++r) {
        hsa_signal_store_relaxed(sig, 1);
        double a = now();
        HSACK(hsa_amd_memory_async_copy(dst, da, src, sa, n, 0, nullptr, sig));
        while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                         HSA_WAIT_STATE_BLOCKED) >= 1) {
        }
        if (r >= 0) t += now() - a;
      }
      printf("%s hsa_async_copy          %.1f GB/s\n", dn, reps * n / t / 1e9);
    }
    for (uint32_t e : engines) {
      double t = 0;
      for (int r = -1; r < reps; ++r) {
        hsa_signal_store_relaxed(sig, 1);
        double a = now();
        hsa_status_t st = hsa_amd_memory_async_copy_on_engine(
            dst, da, src, sa, n, 0, nullptr, sig, (hsa_amd_sdma_engine_id_t)e, true);
        if (st != HSA_STATUS_SUCCESS) {
          printf("%s engine 0x%x: refused (%d)\n", dn, e, (int)st);
          t = -1;
          break;
        }
        while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                         HSA_WAIT_STATE_BLOCKED) >= 1) {
        }
        if (r >= 0) t += now() - a;
      }
      if (t > 0) printf("%s engine 0x%-4x          %.1f GB/s\n", dn, e, reps * n / t / 1e9);
    }
    // split each copy over k engines
    for (size_t k = 2; k <= engines.size(); k *= 2) {
      double t = 0;
      bool ok = true;
      for (int r = -1; r < reps && ok; ++r) {
        hsa_signal_store_relaxed(sig, (hsa_signal_value_t)k);
        double a = now();
        const size_t part = (n / k + 4095) & ~(size_t)4095;
        for (size_t j = 0; j < k; ++j) {
          size_t off = j * part, len = off >= n ? 0 : (n - off < part ? n - off : part);
          hsa_status_t st = hsa_amd_memory_async_copy_on_engine(
              (char*)dst + off, da, (char*)src + off, sa, len, 0, nullptr, sig,
              (hsa_amd_sdma_engine_id_t)engines[j], true);
          if (st != HSA_STATUS_SUCCESS) {
            printf("%s split %zu: refused (%d)\n", dn, k, (int)st);
            ok = false;
            hsa_signal_subtract_relaxed(sig, (hsa_signal_value_t)(k - j));
            break;
          }
        }
        while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                         HSA_WAIT_STATE_BLOCKED) >= 1) {
        }
        if (r >= 0) t += now() - a;
      }
      if (ok) printf("%s split over %zu engines  %.1f GB/s\n", dn, k, reps * n / t / 1e9);
    }
    // chunked stream: 256 MiB copies queued back to back on one engine (the engine pipeline)
    if (!engines.empty()) {
      const size_t chunk = 256ull << 20;
      size_t nch = (n + chunk - 1) / chunk;
      double t = 0;
      for (int r = -1; r < reps; ++r) {
        hsa_signal_store_relaxed(sig, (hsa_signal_value_t)nch);
        double a = now();
        for (size_t j = 0; j < nch; ++j) {
          size_t off = j * chunk, len = n - off < chunk ? n - off : chunk;
          HSACK(hsa_amd_memory_async_copy_on_engine((char*)dst + off, da, (char*)src + off, sa,
                                                    len, 0, nullptr, sig,
                                                    (hsa_amd_sdma_engine_id_t)engines[0], true));
        }
        while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                         HSA_WAIT_STATE_BLOCKED) >= 1) {
        }
        if (r >= 0) t += now() - a;
      }
      printf("%s 256MiB chunks, 1 engine %.1f GB/s\n", dn, reps * n / t / 1e9);
    }
    hsa_signal_destroy(sig);
  }
  // bidirectional: D2H of one buffer on the preferred D2H engine while H2D of another runs on
  // the preferred H2D engine (the streamed preemption hand-off does exactly this)
  {
    void* dev2 = nullptr;
    HIPCK(hipMalloc(&dev2, n));
    void* host2 = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (thp) madvise(host2, n, MADV_HUGEPAGE);
    memset(host2, 3, n);
    HIPCK(hipHostRegister(host2, n, hipHostRegisterMapped | hipHostRegisterPortable));
    uint32_t de = d2h_pref ? (d2h_pref & (~d2h_pref + 1)) : 1, he = h2d_pref ? (h2d_pref & (~h2d_pref + 1)) : 1;
    if (he == de) he = de << 1;
    hsa_signal_t sa, sb;
    HSACK(hsa_signal_create(1, 0, nullptr, &sa));
    HSACK(hsa_signal_create(1, 0, nullptr, &sb));
    double t = 0;
    for (int r = -1; r < reps; ++r) {
      hsa_signal_store_relaxed(sa, 1);
      hsa_signal_store_relaxed(sb, 1);
      double a0 = now();
      HSACK(hsa_amd_memory_async_copy_on_engine(hdev, ag.cpu, dev, ag.gpu, n, 0, nullptr, sa,
                                                (hsa_amd_sdma_engine_id_t)de, true));
      HSACK(hsa_amd_memory_async_copy_on_engine(dev2, ag.gpu, host2, ag.cpu, n, 0, nullptr, sb,
                                                (hsa_amd_sdma_engine_id_t)he, true));
      while (hsa_signal_wait_scacquire(sa, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                       HSA_WAIT_STATE_BLOCKED) >= 1) {
      }
      while (hsa_signal_wait_scacquire(sb, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                       HSA_WAIT_STATE_BLOCKED) >= 1) {
      }
      if (r >= 0) t += now() - a0;
    }
    printf("bidir d2h(0x%x)+h2d(0x%x) each %.1f GB/s, aggregate %.1f GB/s\n", de, he,
           reps * n / t / 1e9, 2.0 * reps * n / t / 1e9);
    hsa_signal_destroy(sa);
    hsa_signal_destroy(sb);
    HIPCK(hipHostUnregister(host2));
    munmap(host2, n);
    HIPCK(hipFree(dev2));
  }
  // verify the D2H landed
  HIPCK(hipMemset(dev, 0x5a, n));
  HIPCK(hipDeviceSynchronize());
  {
    hsa_signal_t sig;
    HSACK(hsa_signal_create(1, 0, nullptr, &sig));
    HSACK(hsa_amd_memory_async_copy(hdev, ag.cpu, dev, ag.gpu, n, 0, nullptr, sig));
    hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    const unsigned char* h = (const unsigned char*)host;
    size_t bad = 0;
    for (size_t i = 0; i < n; i += 4093) bad += h[i] != 0x5a;
    printf("verify d2h: %s\n", bad ? "MISMATCH" : "ok");
    hsa_signal_destroy(sig);
  }
  HIPCK(hipStreamDestroy(s));
  HIPCK(hipFree(dev));
  if (reg) {
    HIPCK(hipHostUnregister(host));
    munmap(host, n);
  } else {
    HIPCK(hipHostFree(host));
  }
  hsa_shut_down();
  return 0;
}
