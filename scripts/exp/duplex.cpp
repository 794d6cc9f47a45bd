// Experiment: both directions of the PCIe link at once, with the finish time of each direction
// measured on its own (sdma_copy.cpp's "bidir" line reports only the slower one).  The
// overlapped bench (save streaming out while a restore streams back in) reaches ~63 GB/s out
// and ~45-50 in (raw, TPZ1 0.80 on the wire); this isolates the link from the pipeline.
//
//   hipcc -O2 -std=c++17 scripts/exp/duplex.cpp -lhsa-runtime64 -o scripts/exp/duplex
//   ./duplex [GiB] [thp|shm]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>
#include <string>
#include <thread>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define HIPCK(x)                                                \
  do {                                                          \
    hipError_t e_ = (x);                                        \
    if (e_ != hipSuccess) {                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));   \
      exit(1);                                                  \
    }                                                           \
  } while (0)
#define HSACK(x)                                                \
  do {                                                          \
    if ((x) != HSA_STATUS_SUCCESS) {                            \
      fprintf(stderr, "%s failed\n", #x);                       \
      exit(1);                                                  \
    }                                                           \
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

// Copy kernel for the "kernel" directions: every workgroup moves a contiguous 1 MiB slab with
// dwordx4 loads/stores; reading host-mapped memory turns each load into a PCIe read request
// issued by the CUs (many more outstanding reads than one SDMA engine keeps in flight).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                              size_t n16) {
  const size_t per = (1u << 20) / 16, b = (size_t)blockIdx.x * per;
  const size_t e = b + per < n16 ? b + per : n16;
  for (size_t i = b + threadIdx.x; i < e; i += 256 * 4) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * 256 < e) v[u] = __builtin_nontemporal_load(src + i + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * 256 < e) __builtin_nontemporal_store(v[u], dst + i + u * 256);
  }
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// kind "thp": private anonymous memory with transparent huge pages; "shm": a /dev/shm file
// mapping (what a spill region shared with a successor process is: 4 KiB pages unless the
// kernel enables shmem THP)
static std::string g_kind = "thp";

static void* pinned(size_t n, int fill) {
  void* p;
  if (g_kind == "shm") {
    char name[64];
    snprintf(name, sizeof(name), "/dev/shm/duplex-%d-%d", (int)getpid(), fill);
    int fd = open(name, O_RDWR | O_CREAT | O_TRUNC, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)n)) exit(1);
    unlink(name);
    p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
  } else {
    p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  }
  if (p == MAP_FAILED) exit(1);
  madvise(p, n, MADV_HUGEPAGE);
  memset(p, fill, n);
  HIPCK(hipHostRegister(p, n, hipHostRegisterMapped | hipHostRegisterPortable));
  return p;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 2.0;
  if (argc > 2) g_kind = argv[2];
  printf("host memory: %s\n", g_kind.c_str());
  const size_t n = (size_t)(gib * (1ull << 30));
  const size_t chunk = 256ull << 20;
  HIPCK(hipSetDevice(0));
  hipDeviceProp_t p;
  HIPCK(hipGetDeviceProperties(&p, 0));
  Agents ag;
  ag.bdf = (uint32_t)((p.pciBusID << 8) | (p.pciDeviceID << 3));
  HSACK(hsa_init());
  HSACK(hsa_iterate_agents(find_gpu, &ag));
  if (!ag.found) return 1;
  void *dev_out, *dev_in;
  HIPCK(hipMalloc(&dev_out, n));
  HIPCK(hipMalloc(&dev_in, n));
  HIPCK(hipMemset(dev_out, 7, n));
  void* host_out = pinned(n, 1);
  void* host_in = pinned(n, 3);
  void *hd_out, *hd_in;
  HIPCK(hipHostGetDevicePointer(&hd_out, host_out, 0));
  HIPCK(hipHostGetDevicePointer(&hd_in, host_in, 0));
  hipStream_t s;
  HIPCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipStream_t s2, s3;
  HIPCK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  HIPCK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
  hipEvent_t ev, ev2, ev3;
  HIPCK(hipEventCreateWithFlags(&ev3, hipEventDisableTiming));
  HIPCK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPCK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
  hsa_signal_t so, si;
  HSACK(hsa_signal_create(1, 0, nullptr, &so));
  HSACK(hsa_signal_create(1, 0, nullptr, &si));
  const size_t nch = (n + chunk - 1) / chunk;

  // out: D2H on SDMA engine `de` (0 = none, KOUT = copy kernel); in: H2D on SDMA engine
  // `he`, or via hipMemcpyAsync when he == 0 (what the restore uses), KIN = copy kernel,
  // TWO = SDMA engines 0 and 1 taking alternate halves of each chunk, none when he == -1.
  const uint32_t KOUT = 0x100;
  const int KIN = -2, TWO = -3, HIP2 = -4;  // HIP2: hipMemcpyAsync halves on two streams
  auto run = [&](uint32_t de, int he, const char* label) {
    double to_sum = 0, ti_sum = 0;
    const int reps = 4;
    for (int r = -1; r < reps; ++r) {
      hsa_signal_store_relaxed(so, de && de != KOUT ? (hsa_signal_value_t)nch : 0);
      hsa_signal_store_relaxed(si, he > 0 ? (hsa_signal_value_t)nch : he == TWO ? (hsa_signal_value_t)(2 * nch) : 0);
      const double t0 = now();
      for (size_t j = 0; j < nch; ++j) {
        const size_t off = j * chunk, len = n - off < chunk ? n - off : chunk;
        if (de == KOUT)
          hipLaunchKernelGGL(k_copy, dim3((unsigned)((len + (1u << 20) - 1) >> 20)), dim3(256), 0, s2,
                             (const u32x4*)((char*)dev_out + off), (u32x4*)((char*)hd_out + off), len / 16);
        else if (de)
          HSACK(hsa_amd_memory_async_copy_on_engine((char*)hd_out + off, ag.cpu,
                                                    (char*)dev_out + off, ag.gpu, len, 0,
                                                    nullptr, so, (hsa_amd_sdma_engine_id_t)de,
                                                    true));
        if (he > 0)
          HSACK(hsa_amd_memory_async_copy_on_engine((char*)dev_in + off, ag.gpu,
                                                    (char*)hd_in + off, ag.cpu, len, 0, nullptr,
                                                    si, (hsa_amd_sdma_engine_id_t)he, true));
        else if (he == 0)
          HIPCK(hipMemcpyAsync((char*)dev_in + off, (char*)host_in + off, len,
                               hipMemcpyHostToDevice, s));
        else if (he == KIN)
          hipLaunchKernelGGL(k_copy, dim3((unsigned)((len + (1u << 20) - 1) >> 20)), dim3(256), 0, s,
                             (const u32x4*)((char*)hd_in + off), (u32x4*)((char*)dev_in + off), len / 16);
        else if (he == HIP2) {
          const size_t h = len / 2;
          HIPCK(hipMemcpyAsync((char*)dev_in + off, (char*)host_in + off, h,
                               hipMemcpyHostToDevice, s));
          HIPCK(hipMemcpyAsync((char*)dev_in + off + h, (char*)host_in + off + h, len - h,
                               hipMemcpyHostToDevice, s3));
        } else if (he == TWO) {
          const size_t h = len / 2;
          HSACK(hsa_amd_memory_async_copy_on_engine((char*)dev_in + off, ag.gpu, (char*)hd_in + off,
                                                    ag.cpu, h, 0, nullptr, si,
                                                    (hsa_amd_sdma_engine_id_t)0x1, true));
          HSACK(hsa_amd_memory_async_copy_on_engine((char*)dev_in + off + h, ag.gpu,
                                                    (char*)hd_in + off + h, ag.cpu, len - h, 0,
                                                    nullptr, si, (hsa_amd_sdma_engine_id_t)0x2, true));
        }
      }
      if (he == 0 || he == KIN || he == HIP2) HIPCK(hipEventRecord(ev, s));
      if (he == HIP2) {  // ev: both halves
        HIPCK(hipEventRecord(ev3, s3));
        HIPCK(hipStreamWaitEvent(s, ev3, 0));
        HIPCK(hipEventRecord(ev, s));
      }
      if (de == KOUT) HIPCK(hipEventRecord(ev2, s2));
      double t_out = de ? 0 : t0, t_in = he == -1 ? t0 : 0;
      while (!t_out || !t_in) {
        if (!t_out && (de == KOUT ? hipEventQuery(ev2) == hipSuccess
                                  : hsa_signal_load_scacquire(so) < 1))
          t_out = now();
        if (!t_in) {
          if (he > 0 || he == TWO ? hsa_signal_load_scacquire(si) < 1
                                  : hipEventQuery(ev) == hipSuccess)
            t_in = now();
        }
      }
      if (r >= 0) {
        to_sum += t_out - t0;
        ti_sum += t_in - t0;
      }
    }
    printf("%-44s out %6.1f GB/s  in %6.1f GB/s\n", label,
           de ? reps * n / to_sum / 1e9 : 0.0, he != -1 ? reps * n / ti_sum / 1e9 : 0.0);
  };
  // "chase": what the overlapped bench does -- the H2D of chunk j reads the bytes the D2H of
  // chunk j just wrote into the same host buffer, as soon as that copy has completed.
  auto chase = [&](uint32_t de, int he, const char* label) {
    double to_sum = 0, ti_sum = 0;
    const int reps = 4;
    for (int r = -1; r < reps; ++r) {
      hsa_signal_store_relaxed(so, (hsa_signal_value_t)nch);
      hsa_signal_store_relaxed(si, he > 0 ? (hsa_signal_value_t)nch : 0);
      const double t0 = now();
      double t_in = 0;
      std::thread reader([&] {
        for (size_t j = 0; j < nch; ++j) {
          const size_t off = j * chunk, len = n - off < chunk ? n - off : chunk;
          while (hsa_signal_load_scacquire(so) > (hsa_signal_value_t)(nch - j - 1)) {
          }
          if (he > 0)
            HSACK(hsa_amd_memory_async_copy_on_engine((char*)dev_in + off, ag.gpu,
                                                      (char*)hd_out + off, ag.cpu, len, 0,
                                                      nullptr, si, (hsa_amd_sdma_engine_id_t)he,
                                                      true));
          else
            HIPCK(hipMemcpyAsync((char*)dev_in + off, (char*)host_out + off, len,
                                 hipMemcpyHostToDevice, s));
        }
        if (he > 0) {
          while (hsa_signal_load_scacquire(si) >= 1) {
          }
        } else {
          HIPCK(hipStreamSynchronize(s));
        }
        t_in = now();
      });
      for (size_t j = 0; j < nch; ++j) {
        const size_t off = j * chunk, len = n - off < chunk ? n - off : chunk;
        HSACK(hsa_amd_memory_async_copy_on_engine((char*)hd_out + off, ag.cpu,
                                                  (char*)dev_out + off, ag.gpu, len, 0, nullptr,
                                                  so, (hsa_amd_sdma_engine_id_t)de, true));
      }
      while (hsa_signal_load_scacquire(so) >= 1) {
      }
      const double t_out = now();
      reader.join();
      if (r >= 0) {
        to_sum += t_out - t0;
        ti_sum += t_in - t0;
      }
    }
    printf("%-44s out %6.1f GB/s  in %6.1f GB/s (in: from its own start)\n", label,
           reps * n / to_sum / 1e9, reps * n / ti_sum / 1e9);
  };
  if (argc > 3 && std::string(argv[3]) == "kernels") {  // the kernel-copy variants only
    run(0, HIP2, "H2D hipMemcpyAsync x2 streams alone");
    run(0x4, HIP2, "D2H engine 2 + H2D hipMemcpyAsync x2 streams");
    run(0x4, 0, "D2H engine 2 + H2D hipMemcpyAsync");
    run(0x4, TWO, "D2H engine 2 + H2D engines 0+1");
    run(0x8, TWO, "D2H engine 3 + H2D engines 0+1");
    if (argc > 4) return 0;
    run(0, KIN, "H2D kernel alone");
    run(KOUT, -1, "D2H kernel alone");
    run(0, TWO, "H2D engines 0+1 alone");
    run(0x4, 0, "D2H engine 2 + H2D hipMemcpyAsync");
    run(0x4, KIN, "D2H engine 2 + H2D kernel");
    run(0x4, TWO, "D2H engine 2 + H2D engines 0+1");
    run(KOUT, 0x2, "D2H kernel + H2D engine 1");
    run(KOUT, KIN, "D2H kernel + H2D kernel");
    return 0;
  }
  chase(0x4, 0, "chase: D2H engine 2 -> H2D hipMemcpyAsync");
  chase(0x4, 0x2, "chase: D2H engine 2 -> H2D engine 1");
  run(0x4, -1, "D2H engine 2 alone");
  run(0, 0, "H2D hipMemcpyAsync alone");
  run(0, 0x2, "H2D engine 1 alone");
  run(0x4, 0, "D2H engine 2 + H2D hipMemcpyAsync");
  run(0x4, 0x2, "D2H engine 2 + H2D engine 1");
  run(0x8, 0x2, "D2H engine 3 + H2D engine 1");
  run(0x4, 0x1, "D2H engine 2 + H2D engine 0");
  run(0x2, 0x8, "D2H engine 1 + H2D engine 3");
  return 0;
}
