// Experiment: CRC32C-only tile kernel with the lookup tables replicated K times in LDS.
//
// The production kernel (csrc/hip/kernels.hip k_stream_crc<MODE_CRC>) reads 20 table entries
// per 16-byte word from one copy of the tables; the entry index is a data byte, so the 32
// lanes of a ds_read_b32 group hit random banks (bank = dword address mod 32) and each group
// costs ~3.5 LDS cycles instead of 1.  With K copies interleaved (entry e of copy c at dword
// e*K + c) and lane l reading copy l % K, lanes that share a copy can only collide on the
// 32/K banks of their copy, so the expected group cost falls towards 1 as K grows -- at K
// times the LDS footprint.  Same math as production: lane-parallel Horner over 4 KiB rows,
// shift to the tile end, workgroup XOR reduce.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/crc_lds.hip -o scripts/exp/crc_lds
//   ./crc_lds [GB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../csrc/common/crc32c.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define WG 256

template <int K>
__device__ static inline uint32_t look(const uint32_t* s, int t, uint32_t v) {
  return s[(t * 256 + v) * K];
}

template <int K>
__device__ static inline uint32_t raw16(const uint32_t* s, u32x4 w) {
  uint32_t c;
  c = look<K>(s, 15, w.x & 0xff) ^ look<K>(s, 14, (w.x >> 8) & 0xff) ^
      look<K>(s, 13, (w.x >> 16) & 0xff) ^ look<K>(s, 12, w.x >> 24);
  c ^= look<K>(s, 11, w.y & 0xff) ^ look<K>(s, 10, (w.y >> 8) & 0xff) ^
       look<K>(s, 9, (w.y >> 16) & 0xff) ^ look<K>(s, 8, w.y >> 24);
  c ^= look<K>(s, 7, w.z & 0xff) ^ look<K>(s, 6, (w.z >> 8) & 0xff) ^
       look<K>(s, 5, (w.z >> 16) & 0xff) ^ look<K>(s, 4, w.z >> 24);
  c ^= look<K>(s, 3, w.w & 0xff) ^ look<K>(s, 2, (w.w >> 8) & 0xff) ^
       look<K>(s, 1, (w.w >> 16) & 0xff) ^ look<K>(s, 0, w.w >> 24);
  return c;
}

template <int KR>
__device__ static inline uint32_t shift_row(const uint32_t* r, uint32_t a) {
  return look<KR>(r, 0, a & 0xff) ^ look<KR>(r, 1, (a >> 8) & 0xff) ^
         look<KR>(r, 2, (a >> 16) & 0xff) ^ look<KR>(r, 3, a >> 24);
}

// Byte-offset form for K = 1: ((w >> 8k) & 0xff) << 2 is one SDWA shift (src_sel BYTE_k) on
// gfx9-family ISA instead of a bfe + lshl_add pair.
__device__ static inline uint32_t lk(const uint32_t* s, int t, uint32_t w, int k) {
  const uint32_t off = ((w >> (8 * k)) & 0xffu) << 2;
  return *(const uint32_t*)((const char*)s + t * 1024 + off);
}
__device__ static inline uint32_t raw16b(const uint32_t* s, u32x4 w) {
  uint32_t c;
  c = lk(s, 15, w.x, 0) ^ lk(s, 14, w.x, 1) ^ lk(s, 13, w.x, 2) ^ lk(s, 12, w.x, 3);
  c ^= lk(s, 11, w.y, 0) ^ lk(s, 10, w.y, 1) ^ lk(s, 9, w.y, 2) ^ lk(s, 8, w.y, 3);
  c ^= lk(s, 7, w.z, 0) ^ lk(s, 6, w.z, 1) ^ lk(s, 5, w.z, 2) ^ lk(s, 4, w.z, 3);
  c ^= lk(s, 3, w.w, 0) ^ lk(s, 2, w.w, 1) ^ lk(s, 1, w.w, 2) ^ lk(s, 0, w.w, 3);
  return c;
}
__device__ static inline uint32_t shift_rowb(const uint32_t* r, uint32_t a) {
  return lk(r, 0, a, 0) ^ lk(r, 1, a, 1) ^ lk(r, 2, a, 2) ^ lk(r, 3, a, 3);
}

// K copies of the 16 slice tables, KR copies of the 4 row tables; persistent grid-stride loop
// over tiles (the tables are staged once per workgroup).
template <int K, int KR, int UNROLL, bool BYTEOFF = false>
__global__ __launch_bounds__(WG) void k_crc(const uint8_t* __restrict__ buf, uint64_t len,
                                            uint64_t tile, const tpi_crc_tables* __restrict__ T,
                                            uint32_t* __restrict__ crcs, uint32_t init_full) {
  extern __shared__ uint32_t lds[];
  uint32_t* s_slice = lds;
  uint32_t* s_row = lds + 16 * 256 * K;
  uint32_t* s_red = s_row + 4 * 256 * KR;
  const int lane = threadIdx.x;
  for (int i = lane; i < 16 * 256 * K; i += WG) s_slice[i] = (&T->slice[0][0])[i / K];
  for (int i = lane; i < 4 * 256 * KR; i += WG) s_row[i] = (&T->row[0][0])[i / KR];
  __syncthreads();
  const uint32_t* sl = s_slice + (lane % K);
  const uint32_t* rl = s_row + (lane % KR);
  const uint64_t ntiles = len / tile;
  const uint64_t rows = tile / TPI_ROW_BYTES;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint8_t* tb = buf + t * tile;
    uint32_t acc = 0;
    for (uint64_t row = 0; row < rows; row += UNROLL) {
      u32x4 w[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
        w[u] = __builtin_nontemporal_load(
            (const u32x4*)(tb + (row + u) * TPI_ROW_BYTES + lane * 16));
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        if (BYTEOFF) acc = shift_rowb(rl, acc) ^ raw16b(sl, w[u]);
        else acc = shift_row<KR>(rl, acc) ^ raw16<K>(sl, w[u]);
      }
    }
    uint32_t contrib = tpi_multmodp(T->lane_shift[lane], acc);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) contrib ^= __shfl_xor(contrib, o, 64);
    __syncthreads();  // s_red reuse across tiles
    if ((lane & 63) == 0) s_red[lane >> 6] = contrib;
    __syncthreads();
    if (lane == 0) crcs[t] = s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3] ^ init_full ^ 0xFFFFFFFFu;
  }
}

static uint32_t crc_bitwise(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (TPI_CRC32C_POLY & (0u - (c & 1)));
  }
  return c ^ 0xFFFFFFFFu;
}

template <int K, int KR, int UNROLL, bool BYTEOFF = false>
static void run(const char* name, const uint8_t* d, uint64_t n, uint64_t tile,
                const tpi_crc_tables* dt, uint32_t* dcrc, uint32_t init, int grid_per_cu,
                std::vector<uint32_t>* out) {
  const size_t lds = (16 * 256 * K + 4 * 256 * KR + 4) * 4;
  auto kern = k_crc<K, KR, UNROLL, BYTEOFF>;
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const uint64_t ntiles = n / tile;
  const unsigned grid = (unsigned)std::min<uint64_t>(ntiles, (uint64_t)p.multiProcessorCount * grid_per_cu);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(WG), lds, 0, d, n, tile, dt, dcrc, init);
  CK(hipDeviceSynchronize());
  const int iters = 10;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL(kern, dim3(grid), dim3(WG), lds, 0, d, n, tile, dt, dcrc, init);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  out->assign(ntiles, 0);
  CK(hipMemcpy(out->data(), dcrc, ntiles * 4, hipMemcpyDeviceToHost));
  printf("%-28s LDS %6zu B  grid %6u  %7.1f GB/s\n", name, lds, grid,
         (double)n * iters / (ms * 1e-3) / 1e9);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 8.0;
  const uint64_t tile = 1 << 20;
  const uint64_t n = (uint64_t)(gb * 1e9) / tile * tile;
  tpi_crc_tables* ht = new tpi_crc_tables;
  tpi_crc_tables_init(ht);
  const uint32_t init = tpi_multmodp(tpi_x8nmodp(tile, ht->x2n), 0xFFFFFFFFu);
  tpi_crc_tables* dt;
  CK(hipMalloc(&dt, sizeof(*ht)));
  CK(hipMemcpy(dt, ht, sizeof(*ht), hipMemcpyHostToDevice));
  uint8_t* d;
  CK(hipMalloc(&d, n));
  std::vector<uint8_t> h(tile * 2);
  srand(7);
  for (auto& x : h) x = (uint8_t)rand();
  for (uint64_t off = 0; off < n; off += h.size())
    CK(hipMemcpy(d + off, h.data(), std::min<uint64_t>(h.size(), n - off), hipMemcpyHostToDevice));
  uint32_t* dcrc;
  CK(hipMalloc(&dcrc, (n / tile) * 4));
  const uint32_t want0 = crc_bitwise(h.data(), tile), want1 = crc_bitwise(h.data() + tile, tile);
  std::vector<uint32_t> ref, got;
  run<1, 1, 8>("K=1 KR=1 U=8 (production)", d, n, tile, dt, dcrc, init, 8, &ref);
  bool ok = ref[0] == want0 && ref[1] == want1;
  printf("  reference tiles vs bitwise: %s\n", ok ? "ok" : "MISMATCH");
#define V(K, KR, U, G)                                                          \
  run<K, KR, U>("K=" #K " KR=" #KR " U=" #U " g=" #G, d, n, tile, dt, dcrc, init, G, &got); \
  if (got != ref) { printf("  MISMATCH\n"); ok = false; }
  run<1, 1, 8, true>("K=1 byte-offset U=8", d, n, tile, dt, dcrc, init, 8, &got);
  if (got != ref) { printf("  MISMATCH\n"); ok = false; }
  run<1, 1, 16, true>("K=1 byte-offset U=16", d, n, tile, dt, dcrc, init, 8, &got);
  if (got != ref) { printf("  MISMATCH\n"); ok = false; }
  V(1, 1, 16, 8)
  V(2, 2, 8, 4)
  V(2, 2, 16, 4)
  V(4, 4, 8, 2)
  V(4, 4, 16, 2)
  V(4, 2, 16, 2)
  V(8, 4, 8, 1)
  V(8, 4, 16, 1)
  V(8, 1, 16, 1)
  printf("%s\n", ok ? "all variants match" : "MISMATCH");
  return ok ? 0 : 1;
}
