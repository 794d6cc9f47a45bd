// Round 5 experiment: which HBM copy pattern moves the most bytes on MI355X?  The hand-off's
// fused copy (k_stream_hash<HASH_COPY>) reaches 5.27 TB/s of traffic with its digest; this
// times the bare access patterns it could use, without hashing or segment lookups:
//   rows      : one 256-lane workgroup per 1 MiB tile, 16 B per lane per 4 KiB row, U rows
//               in flight (the hand-off kernel's layout)
//   wide      : the same with 32 B per lane (two adjacent 16 B words) per 8 KiB row
//   persist   : a grid of 8 x 256 workgroups striding over the tiles
// each with non-temporal (nt) or ordinary (ld/st) loads and stores, plus hipMemcpyAsync D2D.
//   hipcc --offload-arch=gfx950 -O3 -o copy_variants copy_variants.hip
//   ./copy_variants [GB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int WG = 256;
constexpr uint64_t TILE = 1 << 20;

template <bool NTL>
__device__ inline u32x4 ld(const u32x4* p) {
  if (NTL) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NTS>
__device__ inline void st(u32x4* p, u32x4 v) {
  if (NTS)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// 16 B per lane per 4 KiB row, U rows in flight; one workgroup per tile
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(WG) void k_rows(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                             uint64_t n16) {
  const uint64_t base = (uint64_t)blockIdx.x * (TILE / 16) + threadIdx.x;
  const uint64_t rows = TILE / 4096;
  for (uint64_t r = 0; r < rows; r += U) {
    u32x4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (r + u) * WG;
      w[u] = i < n16 ? ld<NTL>(src + i) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (r + u) * WG;
      if (i < n16) st<NTS>(dst + i, w[u]);
    }
  }
}

// 32 B per lane per 8 KiB row
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(WG) void k_wide(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                             uint64_t n16) {
  const uint64_t base = (uint64_t)blockIdx.x * (TILE / 16) + 2 * threadIdx.x;
  const uint64_t rows = TILE / 8192;
  for (uint64_t r = 0; r < rows; r += U) {
    u32x4 w[2 * U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (r + u) * 2 * WG;
      w[2 * u] = i < n16 ? ld<NTL>(src + i) : u32x4{0, 0, 0, 0};
      w[2 * u + 1] = i + 1 < n16 ? ld<NTL>(src + i + 1) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + (r + u) * 2 * WG;
      if (i < n16) st<NTS>(dst + i, w[2 * u]);
      if (i + 1 < n16) st<NTS>(dst + i + 1, w[2 * u + 1]);
    }
  }
}

// a resident grid striding over the tiles
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(WG) void k_persist(const u32x4* __restrict__ src,
                                                u32x4* __restrict__ dst, uint64_t n16,
                                                uint64_t ntiles) {
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t base = t * (TILE / 16) + threadIdx.x;
    for (uint64_t r = 0; r < TILE / 4096; r += U) {
      u32x4 w[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + (r + u) * WG;
        w[u] = i < n16 ? ld<NTL>(src + i) : u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + (r + u) * WG;
        if (i < n16) st<NTS>(dst + i, w[u]);
      }
    }
  }
}

template <typename F>
static double time_ms(F launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int i = 0; i < 5; ++i) {
    CK(hipEventRecord(a, 0));
    launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float t = 0;
    CK(hipEventElapsedTime(&t, a, b));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms[2];
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 32.0;
  const uint64_t bytes = (uint64_t)(gb * 1e9) / TILE * TILE;
  const uint64_t n16 = bytes / 16, ntiles = bytes / TILE;
  u32x4 *src, *dst;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMemset(src, 0x5a, bytes));
  CK(hipMemset(dst, 0, bytes));
  CK(hipDeviceSynchronize());
  auto report = [&](const char* name, double ms) {
    printf("{\"case\": \"%s\", \"gb\": %.1f, \"ms\": %.3f, \"copy_TBps\": %.3f, \"hbm_traffic_TBps\": %.3f}\n",
           name, bytes / 1e9, ms, bytes / ms / 1e9, 2.0 * bytes / ms / 1e9);
    fflush(stdout);
  };
  report("hipMemcpyAsync D2D", time_ms([&] { CK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, 0)); }));
#define ROWS(U, L, S)                                                                          \
  report("rows U=" #U " load=" #L " store=" #S, time_ms([&] {                                  \
           hipLaunchKernelGGL((k_rows<U, L, S>), dim3(ntiles), dim3(WG), 0, 0, src, dst, n16); \
         }))
  ROWS(2, true, true);
  ROWS(2, false, true);
  ROWS(2, true, false);
  ROWS(2, false, false);
  ROWS(4, true, true);
  ROWS(1, true, true);
#define WIDE(U, L, S)                                                                          \
  report("wide U=" #U " load=" #L " store=" #S, time_ms([&] {                                  \
           hipLaunchKernelGGL((k_wide<U, L, S>), dim3(ntiles), dim3(WG), 0, 0, src, dst, n16); \
         }))
  WIDE(1, true, true);
  WIDE(2, true, true);
  WIDE(2, false, false);
#define PERSIST(U, L, S, G)                                                                     \
  report("persist grid=" #G " U=" #U " load=" #L " store=" #S, time_ms([&] {                    \
           hipLaunchKernelGGL((k_persist<U, L, S>), dim3(G), dim3(WG), 0, 0, src, dst, n16, ntiles); \
         }))
  PERSIST(2, true, true, 2048);
  PERSIST(2, true, true, 4096);
  PERSIST(4, true, true, 2048);
  // sanity: the last copy is complete
  std::vector<unsigned> tail(1024);
  CK(hipMemcpy(tail.data(), (const char*)dst + bytes - 4096, 4096, hipMemcpyDeviceToHost));
  for (unsigned v : tail)
    if (v != 0x5a5a5a5au) {
      fprintf(stderr, "copy incomplete\n");
      return 1;
    }
  CK(hipFree(src));
  CK(hipFree(dst));
  return 0;
}
