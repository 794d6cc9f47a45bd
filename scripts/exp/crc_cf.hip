// Experiment: bank-conflict-free CRC32C tile kernel ("column tables").
//
// crc_lds_round2.md showed the CRC-only kernel is bound by LDS bank conflicts: the table
// index is a data byte, so the 32 lanes of a ds_read_b32 group land on random banks
// (bank = dword mod 32) and a group costs ~3.5 cycles instead of 1.  Replicating whole
// tables per lane does not fit.  Here every table copy lives in ONE bank column instead:
// entry e of column c is dword e*32 + c, so a lookup's bank is its column, whatever the data.
//
//   slice region  32 columns, column c holds slice table (c & 15)      32 KiB
//   row region    RC columns, column c holds row-shift table (c & 3)   RC KiB
//
// At unrolled step j of a word, lane l uses column (j + l) mod 32 -- a permutation of the
// 32 banks over a lane group -- and therefore slice table (j + l) mod 16.  Which byte of the
// word that table needs depends on the lane, so each lane first rotates its 16-byte word left
// by (l mod 16) bytes (8 v_cndmask + 4 v_alignbyte, lane-constant masks); then step j always
// reads byte 15 - j.  The row shift does the same with the byte of the accumulator chosen by
// a lane-constant bfe offset.  Same math and result as csrc/hip/kernels.hip k_stream_crc.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/crc_cf.hip -o scripts/exp/crc_cf
//   ./crc_cf --selftest     (host emulation of the lane mapping: results + bank permutation)
//   ./crc_cf [GB]           (GPU: variants vs the production layout, bit-exact check)
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
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

__host__ __device__ static inline uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, s);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (s & 3)));
#endif
}

// Lane-constant part of the mapping.
struct LaneMap {
  bool m1, m2;       // dword rotation by 1 / by 2
  uint32_t s;        // alignbyte shift
  uint32_t colS[16]; // byte offset of the slice column at step j
  uint32_t colR[4];  // byte offset of the row column at step j
  uint32_t shR[4];   // bit offset of the accumulator byte at row step j
};

template <int RC>
__host__ __device__ static inline void lane_map(int lane, LaneMap& m) {
  const int l32 = lane & 31, r = lane & 15;
  const int q2 = ((r + 3) >> 2) & 3;
  m.m1 = q2 & 1;
  m.m2 = q2 & 2;
  m.s = (4 - (r & 3)) & 3;
  for (int j = 0; j < 16; ++j) m.colS[j] = (uint32_t)((j + l32) & 31) * 4;
  for (int j = 0; j < 4; ++j) {
    m.colR[j] = (uint32_t)((j + l32) & (RC - 1)) * 4;
    m.shR[j] = 8u * (uint32_t)((j + l32) & 3);
  }
}

__host__ __device__ static inline void rotate(const LaneMap& m, u32x4 w, uint32_t R[4]) {
  const uint32_t t0 = m.m1 ? w.w : w.x, t1 = m.m1 ? w.x : w.y, t2 = m.m1 ? w.y : w.z,
                 t3 = m.m1 ? w.z : w.w;
  const uint32_t x0 = m.m2 ? t2 : t0, x1 = m.m2 ? t3 : t1, x2 = m.m2 ? t0 : t2,
                 x3 = m.m2 ? t1 : t3;
  R[0] = alignbyte(x1, x0, m.s);
  R[1] = alignbyte(x2, x1, m.s);
  R[2] = alignbyte(x3, x2, m.s);
  R[3] = alignbyte(x0, x3, m.s);
}

__host__ __device__ static inline uint32_t at(const uint32_t* base, uint32_t byte_off) {
  return *(const uint32_t*)((const char*)base + byte_off);
}

__host__ __device__ static inline uint32_t raw16_cf(const uint32_t* s, const LaneMap& m, u32x4 w) {
  uint32_t R[4];
  rotate(m, w, R);
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int pos = 15 - j;
    const uint32_t v = (R[pos >> 2] >> (8 * (pos & 3))) & 0xffu;
    c ^= at(s, v * 128u + m.colS[j]);
  }
  return c;
}

template <int RC>
__host__ __device__ static inline uint32_t shift_row_cf(const uint32_t* r, const LaneMap& m,
                                                        uint32_t a) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) c ^= at(r, ((a >> m.shR[j]) & 0xffu) * (RC * 4u) + m.colR[j]);
  return c;
}

template <int RC>
static void build_cf(const tpi_crc_tables* T, std::vector<uint32_t>& out) {
  out.assign(256 * 32 + 256 * RC, 0);
  for (int e = 0; e < 256; ++e)
    for (int c = 0; c < 32; ++c) out[e * 32 + c] = T->slice[c & 15][e];
  for (int e = 0; e < 256; ++e)
    for (int c = 0; c < RC; ++c) out[256 * 32 + e * RC + c] = T->row[c & 3][e];
}

// ---- perm variant: one v_perm_b32 forms each lookup address ----------------------------------
//
// Rows of 256 B: entry v of a column sits at byte v*256 + column*4, slice columns at bytes
// 0..127, row-shift columns at 128..255 (bank = column either way, 64 KiB in all).  The
// address of a lookup is then (data byte) << 8 | (column byte): v_perm_b32 assembles it from
// the data dword and a register packing four lane columns, so a lookup is 1 VALU + ds_read
// (+ half an xor3), against 1 + ds_read + xor in the production layout.

__host__ __device__ static inline uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(s0, s1, sel);
#else
  const uint64_t c = ((uint64_t)s0 << 32) | s1;
  uint32_t d = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t b = (sel >> (8 * i)) & 0xff;
    const uint32_t v = b < 8 ? (uint32_t)(c >> (8 * b)) & 0xff : b == 12 ? 0 : 0xff;
    d |= v << (8 * i);
  }
  return d;
#endif
}

struct LaneMapP {
  bool m1, m2;
  uint32_t s;
  uint32_t colpack[4];  // byte i of colpack[m]: ((4m + i + l) mod 32) * 4
  uint32_t selR[4];     // row step j: byte0 <- colpack[0] byte j, byte1 <- acc byte (j+l)&3
};

__host__ __device__ static inline void lane_map_p(int lane, LaneMapP& m) {
  const int l32 = lane & 31, r = lane & 15;
  const int q2 = ((r + 3) >> 2) & 3;
  m.m1 = q2 & 1;
  m.m2 = q2 & 2;
  m.s = (4 - (r & 3)) & 3;
  for (int k = 0; k < 4; ++k) {
    uint32_t c = 0;
    for (int i = 0; i < 4; ++i) c |= (uint32_t)(((4 * k + i + l32) & 31) * 4) << (8 * i);
    m.colpack[k] = c;
    m.selR[k] = 0x0C0C0000u | ((4u + (uint32_t)((k + l32) & 3)) << 8) | (uint32_t)k;
  }
}

__host__ __device__ static inline uint32_t raw16_pm(const uint32_t* t, const LaneMapP& mp,
                                                    u32x4 w) {
  LaneMap m;
  m.m1 = mp.m1;
  m.m2 = mp.m2;
  m.s = mp.s;
  uint32_t R[4];
  rotate(m, w, R);
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int pos = 15 - j;
    const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(pos & 3)) << 8) | (uint32_t)(j & 3);
    c ^= at(t, perm(R[pos >> 2], mp.colpack[j >> 2], sel));
  }
  return c;
}

__host__ __device__ static inline uint32_t shift_row_pm(const uint32_t* t, const LaneMapP& m,
                                                        uint32_t a) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) c ^= at(t + 32, perm(a, m.colpack[0], m.selR[j]));
  return c;
}

static void build_pm(const tpi_crc_tables* T, std::vector<uint32_t>& out) {
  out.assign(256 * 64, 0);
  for (int e = 0; e < 256; ++e)
    for (int c = 0; c < 32; ++c) {
      out[e * 64 + c] = T->slice[c & 15][e];
      out[e * 64 + 32 + c] = T->row[c & 3][e];
    }
}

static bool selftest_pm(const tpi_crc_tables* T) {
  std::vector<uint32_t> t;
  build_pm(T, t);
  srand(13);
  bool ok = true;
  for (int it = 0; it < 2000 && ok; ++it) {
    u32x4 w;
    w.x = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    w.y = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    w.z = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    w.w = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    const uint32_t a = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    uint32_t want = 0, wrow = 0;
    const uint8_t* b = (const uint8_t*)&w;
    for (int k = 0; k < 16; ++k) want ^= T->slice[15 - k][b[k]];
    for (int k = 0; k < 4; ++k) wrow ^= T->row[k][(a >> (8 * k)) & 0xff];
    std::set<uint32_t> banks[20];
    for (int lane = 0; lane < 64; ++lane) {
      LaneMapP m;
      lane_map_p(lane, m);
      if (raw16_pm(t.data(), m, w) != want || shift_row_pm(t.data(), m, a) != wrow) {
        printf("selftest perm: lane %d wrong\n", lane);
        ok = false;
        break;
      }
      if (lane < 32) {
        LaneMap mm;
        mm.m1 = m.m1; mm.m2 = m.m2; mm.s = m.s;
        uint32_t R[4];
        rotate(mm, w, R);
        for (int j = 0; j < 16; ++j) {
          const int pos = 15 - j;
          const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(pos & 3)) << 8) | (uint32_t)(j & 3);
          banks[j].insert((perm(R[pos >> 2], m.colpack[j >> 2], sel) / 4) % 32);
        }
        for (int j = 0; j < 4; ++j) banks[16 + j].insert(((128 + perm(a, m.colpack[0], m.selR[j])) / 4) % 32);
      }
    }
    for (int j = 0; j < 20 && ok; ++j)
      if (banks[j].size() != 32) { printf("perm step %d: %zu banks\n", j, banks[j].size()); ok = false; }
  }
  printf("selftest perm: %s\n", ok ? "ok (results exact, all 20 lookups on 32 distinct banks)" : "FAILED");
  return ok;
}

// ---- production layout (K=1), for the timing baseline ------------------------------------------

__device__ static inline uint32_t raw16(const uint32_t* s, u32x4 w) {
  uint32_t c;
  c = s[15 * 256 + (w.x & 0xff)] ^ s[14 * 256 + ((w.x >> 8) & 0xff)] ^
      s[13 * 256 + ((w.x >> 16) & 0xff)] ^ s[12 * 256 + (w.x >> 24)];
  c ^= s[11 * 256 + (w.y & 0xff)] ^ s[10 * 256 + ((w.y >> 8) & 0xff)] ^
       s[9 * 256 + ((w.y >> 16) & 0xff)] ^ s[8 * 256 + (w.y >> 24)];
  c ^= s[7 * 256 + (w.z & 0xff)] ^ s[6 * 256 + ((w.z >> 8) & 0xff)] ^
       s[5 * 256 + ((w.z >> 16) & 0xff)] ^ s[4 * 256 + (w.z >> 24)];
  c ^= s[3 * 256 + (w.w & 0xff)] ^ s[2 * 256 + ((w.w >> 8) & 0xff)] ^
       s[1 * 256 + ((w.w >> 16) & 0xff)] ^ s[0 * 256 + (w.w >> 24)];
  return c;
}

__device__ static inline uint32_t shift_row(const uint32_t* r, uint32_t a) {
  return r[a & 0xff] ^ r[256 + ((a >> 8) & 0xff)] ^ r[512 + ((a >> 16) & 0xff)] ^
         r[768 + (a >> 24)];
}

template <int UNROLL>
__global__ __launch_bounds__(WG) void k_crc_prod(const uint8_t* __restrict__ buf, uint64_t len,
                                                 uint64_t tile, const tpi_crc_tables* __restrict__ T,
                                                 const uint32_t* __restrict__ unused,
                                                 uint32_t* __restrict__ crcs, uint32_t init_full) {
  __shared__ uint32_t lds[20 * 256 + 4];
  uint32_t* s_slice = lds;
  uint32_t* s_row = lds + 16 * 256;
  uint32_t* s_red = lds + 20 * 256;
  const int lane = threadIdx.x;
  for (int i = lane; i < 20 * 256 / 4; i += WG) ((u32x4*)lds)[i] = ((const u32x4*)T)[i];
  __syncthreads();
  const uint64_t ntiles = len / tile, rows = tile / TPI_ROW_BYTES;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint8_t* tb = buf + t * tile;
    uint32_t acc = 0;
    for (uint64_t row = 0; row < rows; row += UNROLL) {
      u32x4 w[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
        w[u] = __builtin_nontemporal_load((const u32x4*)(tb + (row + u) * TPI_ROW_BYTES + lane * 16));
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) acc = shift_row(s_row, acc) ^ raw16(s_slice, w[u]);
    }
    uint32_t contrib = tpi_multmodp(T->lane_shift[lane], acc);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) contrib ^= __shfl_xor(contrib, o, 64);
    __syncthreads();
    if ((lane & 63) == 0) s_red[lane >> 6] = contrib;
    __syncthreads();
    if (lane == 0) crcs[t] = s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3] ^ init_full ^ 0xFFFFFFFFu;
  }
}

// ---- column-table kernel -------------------------------------------------------------------

template <int RC, int UNROLL>
__global__ __launch_bounds__(WG) void k_crc_cf(const uint8_t* __restrict__ buf, uint64_t len,
                                               uint64_t tile, const tpi_crc_tables* __restrict__ T,
                                               const uint32_t* __restrict__ cf,
                                               uint32_t* __restrict__ crcs, uint32_t init_full) {
  extern __shared__ uint32_t lds[];
  uint32_t* s_slice = lds;
  uint32_t* s_row = lds + 256 * 32;
  uint32_t* s_red = s_row + 256 * RC;
  const int lane = threadIdx.x;
  for (int i = lane; i < (256 * 32 + 256 * RC) / 4; i += WG) ((u32x4*)lds)[i] = ((const u32x4*)cf)[i];
  LaneMap m;
  lane_map<RC>(lane, m);
  __syncthreads();
  const uint64_t ntiles = len / tile, rows = tile / TPI_ROW_BYTES;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint8_t* tb = buf + t * tile;
    uint32_t acc = 0;
    for (uint64_t row = 0; row < rows; row += UNROLL) {
      u32x4 w[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
        w[u] = __builtin_nontemporal_load((const u32x4*)(tb + (row + u) * TPI_ROW_BYTES + lane * 16));
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
        acc = shift_row_cf<RC>(s_row, m, acc) ^ raw16_cf(s_slice, m, w[u]);
    }
    uint32_t contrib = tpi_multmodp(T->lane_shift[lane], acc);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) contrib ^= __shfl_xor(contrib, o, 64);
    __syncthreads();
    if ((lane & 63) == 0) s_red[lane >> 6] = contrib;
    __syncthreads();
    if (lane == 0) crcs[t] = s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3] ^ init_full ^ 0xFFFFFFFFu;
  }
}

// WGT threads per workgroup: 256 (one tile at a time) or 512 (two tiles, one per half, sharing
// the 64 KiB of tables -- twice the waves per CU for the same LDS).
template <int UNROLL, int WGT>
__global__ __launch_bounds__(WGT) void k_crc_pm(const uint8_t* __restrict__ buf, uint64_t len,
                                                uint64_t tile, const tpi_crc_tables* __restrict__ T,
                                                const uint32_t* __restrict__ pm,
                                                uint32_t* __restrict__ crcs, uint32_t init_full) {
  __shared__ uint32_t lds[256 * 64 + 8];  // static: a dynamic base costs an add per lookup
  uint32_t* s_red = lds + 256 * 64;
  const int tid = threadIdx.x, lane = tid & 255, half = tid >> 8;
  for (int i = tid; i < 256 * 64 / 4; i += WGT) ((u32x4*)lds)[i] = ((const u32x4*)pm)[i];
  LaneMapP m;
  lane_map_p(lane, m);
  __syncthreads();
  const uint64_t ntiles = len / tile, rows = tile / TPI_ROW_BYTES;
  const int per = WGT / 256;
  for (uint64_t t0 = (uint64_t)blockIdx.x * per; t0 < ntiles; t0 += (uint64_t)gridDim.x * per) {
    const uint64_t t = t0 + half;
    uint32_t contrib = 0;
    if (t < ntiles) {
      const uint8_t* tb = buf + t * tile;
      uint32_t acc = 0;
      for (uint64_t row = 0; row < rows; row += UNROLL) {
        u32x4 w[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
          w[u] = __builtin_nontemporal_load((const u32x4*)(tb + (row + u) * TPI_ROW_BYTES + lane * 16));
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
          acc = shift_row_pm(lds, m, acc) ^ raw16_pm(lds, m, w[u]);
      }
      contrib = tpi_multmodp(T->lane_shift[lane], acc);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) contrib ^= __shfl_xor(contrib, o, 64);
    __syncthreads();
    if ((tid & 63) == 0) s_red[tid >> 6] = contrib;
    __syncthreads();
    if (lane == 0 && t < ntiles) {
      const uint32_t* r = s_red + 4 * half;
      crcs[t] = r[0] ^ r[1] ^ r[2] ^ r[3] ^ init_full ^ 0xFFFFFFFFu;
    }
  }
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

// ---- host ------------------------------------------------------------------------------------

static uint32_t crc_bitwise(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (TPI_CRC32C_POLY & (0u - (c & 1)));
  }
  return c ^ 0xFFFFFFFFu;
}

template <int RC>
static bool selftest(const tpi_crc_tables* T) {
  std::vector<uint32_t> cf;
  build_cf<RC>(T, cf);
  const uint32_t* s = cf.data();
  const uint32_t* r = cf.data() + 256 * 32;
  srand(11);
  bool ok = true;
  for (int it = 0; it < 2000 && ok; ++it) {
    u32x4 w;
    w.x = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    w.y = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    w.z = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    w.w = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    const uint32_t a = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    uint32_t want = 0, wrow = 0;
    const uint8_t* b = (const uint8_t*)&w;
    for (int k = 0; k < 16; ++k) want ^= T->slice[15 - k][b[k]];
    for (int k = 0; k < 4; ++k) wrow ^= T->row[k][(a >> (8 * k)) & 0xff];
    std::set<uint32_t> banks[16], rbanks[4];
    for (int lane = 0; lane < 64; ++lane) {
      LaneMap m;
      lane_map<RC>(lane, m);
      if (raw16_cf(s, m, w) != want || shift_row_cf<RC>(r, m, a) != wrow) {
        printf("selftest RC=%d: lane %d wrong\n", RC, lane);
        ok = false;
        break;
      }
      if (lane < 32) {  // bank of every lookup of the first lane group
        uint32_t R[4];
        rotate(m, w, R);
        for (int j = 0; j < 16; ++j) {
          const int pos = 15 - j;
          const uint32_t v = (R[pos >> 2] >> (8 * (pos & 3))) & 0xffu;
          banks[j].insert(((v * 128u + m.colS[j]) / 4) % 32);
        }
        for (int j = 0; j < 4; ++j)
          rbanks[j].insert(((((a >> m.shR[j]) & 0xffu) * (RC * 4u) + m.colR[j]) / 4) % 32);
      }
    }
    for (int j = 0; j < 16 && ok; ++j)
      if (banks[j].size() != 32) { printf("slice step %d: %zu banks\n", j, banks[j].size()); ok = false; }
    if (RC == 32)
      for (int j = 0; j < 4 && ok; ++j)
        if (rbanks[j].size() != 32) { printf("row step %d: %zu banks\n", j, rbanks[j].size()); ok = false; }
  }
  printf("selftest RC=%d: %s\n", RC, ok ? "ok (results exact, slice lookups on 32 distinct banks)" : "FAILED");
  return ok;
}

typedef void (*kern_t)(const uint8_t*, uint64_t, uint64_t, const tpi_crc_tables*, const uint32_t*,
                       uint32_t*, uint32_t);

static void run(const char* name, kern_t kern, size_t lds, const uint8_t* d, uint64_t n,
                uint64_t tile, const tpi_crc_tables* dt, const uint32_t* dcf, uint32_t* dcrc,
                uint32_t init, int grid_per_cu, std::vector<uint32_t>* out, int wgt = WG) {
  if (lds > 65536)
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const uint64_t ntiles = n / tile;
  const unsigned grid = (unsigned)std::min<uint64_t>((ntiles + wgt / 256 - 1) / (wgt / 256),
                                                     (uint64_t)p.multiProcessorCount * grid_per_cu);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(wgt), lds, 0, d, n, tile, dt, dcf, dcrc, init);
  CK(hipDeviceSynchronize());
  const int iters = 10;
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL(kern, dim3(grid), dim3(wgt), lds, 0, d, n, tile, dt, dcf, dcrc, init);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  out->assign(ntiles, 0);
  CK(hipMemcpy(out->data(), dcrc, ntiles * 4, hipMemcpyDeviceToHost));
  printf("%-30s LDS %6zu B  grid %6u  %7.1f GB/s\n", name, lds, grid,
         (double)n * iters / (ms * 1e-3) / 1e9);
  fflush(stdout);
}

int main(int argc, char** argv) {
  tpi_crc_tables* ht = new tpi_crc_tables;
  tpi_crc_tables_init(ht);
  if (argc > 1 && !strcmp(argv[1], "--selftest")) {
    const bool ok = selftest<32>(ht) & selftest<16>(ht) & selftest_pm(ht);
    return ok ? 0 : 1;
  }
  const double gb = argc > 1 ? atof(argv[1]) : 8.0;
  const uint64_t tile = 1 << 20;
  const uint64_t n = (uint64_t)(gb * 1e9) / tile * tile;
  const uint32_t init = tpi_multmodp(tpi_x8nmodp(tile, ht->x2n), 0xFFFFFFFFu);
  tpi_crc_tables* dt;
  CK(hipMalloc(&dt, sizeof(*ht)));
  CK(hipMemcpy(dt, ht, sizeof(*ht), hipMemcpyHostToDevice));
  std::vector<uint32_t> cf32, cf16;
  build_cf<32>(ht, cf32);
  build_cf<16>(ht, cf16);
  uint32_t *dcf32, *dcf16;
  CK(hipMalloc(&dcf32, cf32.size() * 4));
  CK(hipMalloc(&dcf16, cf16.size() * 4));
  CK(hipMemcpy(dcf32, cf32.data(), cf32.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcf16, cf16.data(), cf16.size() * 4, hipMemcpyHostToDevice));
  uint8_t* d;
  CK(hipMalloc(&d, n));
  std::vector<uint8_t> h(tile * 2);
  if (getenv("CRC_CF_PATTERN")) {  // a 2-tile pattern repeated (the first measurements)
    srand(7);
    for (auto& x : h) x = (uint8_t)rand();
    for (uint64_t off = 0; off < n; off += h.size())
      CK(hipMemcpy(d + off, h.data(), std::min<uint64_t>(h.size(), n - off), hipMemcpyHostToDevice));
  } else {  // every byte distinct-random (splitmix64 of the word index)
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t*)d, n / 8);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, h.size(), hipMemcpyDeviceToHost));
  }
  uint32_t* dcrc;
  CK(hipMalloc(&dcrc, (n / tile) * 4));
  const uint32_t want0 = crc_bitwise(h.data(), tile), want1 = crc_bitwise(h.data() + tile, tile);
  std::vector<uint32_t> ref, got;
  run("production K=1 U=8 g=8", k_crc_prod<8>, 0, d, n, tile, dt, nullptr, dcrc, init, 8, &ref);
  bool ok = ref[0] == want0 && ref[1] == want1;
  printf("  reference tiles vs bitwise: %s\n", ok ? "ok" : "MISMATCH");
  const size_t l32 = (256 * 32 + 256 * 32 + 4) * 4, l16 = (256 * 32 + 256 * 16 + 4) * 4;
#define V(RC, U, G)                                                                          \
  run("cf RC=" #RC " U=" #U " g=" #G, k_crc_cf<RC, U>, RC == 32 ? l32 : l16, d, n, tile, dt, \
      RC == 32 ? dcf32 : dcf16, dcrc, init, G, &got);                                        \
  if (got != ref) {                                                                          \
    printf("  MISMATCH\n");                                                                  \
    ok = false;                                                                              \
  }
  std::vector<uint32_t> pmt;
  build_pm(ht, pmt);
  uint32_t* dpm;
  CK(hipMalloc(&dpm, pmt.size() * 4));
  CK(hipMemcpy(dpm, pmt.data(), pmt.size() * 4, hipMemcpyHostToDevice));
  const size_t lpm = 0;  // static LDS
#define P(U, W, G)                                                                           \
  run("perm U=" #U " wg=" #W " g=" #G, k_crc_pm<U, W>, lpm, d, n, tile, dt, dpm, dcrc, init, \
      G, &got, W);                                                                           \
  if (got != ref) {                                                                          \
    printf("  MISMATCH\n");                                                                  \
    ok = false;                                                                              \
  }
  P(8, 256, 2)
  P(16, 256, 2)
  P(8, 512, 2)
  P(16, 512, 2)
  P(4, 512, 2)
  V(32, 8, 2)
  V(32, 16, 2)
  V(32, 4, 2)
  V(16, 8, 3)
  V(16, 16, 3)
  V(16, 4, 3)
  V(32, 8, 4)
  V(16, 8, 6)
  // The production entry point (libtpi_hip.so tpi_crc32c_tiles -> k_crc_tiles), same buffer.
  if (void* lib = dlopen("terraform_provider_iterative_amd/_lib/libtpi_hip.so", RTLD_NOW)) {
    typedef int (*fn_t)(const void*, uint64_t, uint64_t, uint32_t*, uint64_t);
    fn_t fn = (fn_t)dlsym(lib, "tpi_crc32c_tiles");
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    fn(d, n, tile, dcrc, 0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < 10; ++i) fn(d, n, tile, dcrc, 0);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    got.assign(n / tile, 0);
    CK(hipMemcpy(got.data(), dcrc, got.size() * 4, hipMemcpyDeviceToHost));
    printf("%-30s %7.1f GB/s%s\n", "libtpi_hip tpi_crc32c_tiles", (double)n * 10 / (ms * 1e-3) / 1e9,
           got == ref ? "" : "  MISMATCH");
    ok = ok && got == ref;
  } else {
    printf("libtpi_hip.so not loaded: %s\n", dlerror());
  }
  printf("%s\n", ok ? "all variants match" : "MISMATCH");
  return ok ? 0 : 1;
}
