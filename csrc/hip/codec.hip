// CDNA4 kernels of the TPZ1 byte-plane checkpoint codec (format: csrc/common/tpz.h).
//
// The checkpoint spill is PCIe-bound (~56 GB/s per GPU) while HBM streams at >5 TB/s, so the
// GPU spends a few hundred microseconds per 256 MiB chunk shrinking what crosses the link:
//
//   k_tpz_analyze  one 256-thread workgroup per tile: sampled 4x256-bin histogram in LDS,
//                  top-15 dictionary per plane (one wave per plane, wave64 max-reductions),
//                  Huffman code lengths of dictionary + escape (one lane per plane, LDS
//                  workspace), exact costs of every mode over the whole tile (lane s also sums
//                  the HUF bits of substream s), cheapest mode per plane -> header + size.
//   k_tpz_encode   one workgroup per tile: blob offset = sum of the earlier tiles' sizes of
//                  the chunk, then rounds of 256 groups (a group = 128 tile bytes, one lane,
//                  8 x dwordx4 loads): DICT codes are fixed-width so they are stored directly;
//                  escapes get their position from a workgroup exclusive scan of 4 packed
//                  16-bit counters (one u64 scan per round); a HUF plane appends the group's
//                  codes to the lane's own substream (start = scan of the analyzed sizes).
//   k_tpz_decode   the inverse, writing whole 128-byte groups of the raw tile; a HUF plane is
//                  decoded by each lane from its own substream through a 2^11-entry LDS table.
//
// Every DICT mode is a template (K = code width) so the 32-code group loops are fully
// unrolled and the code words stay in registers (no scratch).
#include <hip/hip_runtime.h>

#include "../common/tpz.h"
#include "sysmem.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define CWG 256
static_assert(CWG == TPZ_HUF_STREAMS, "HUF substream s is lane s of the codec workgroup");

__device__ static inline uint64_t cmin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// Exclusive scan of one u64 per thread over the workgroup; returns the prefix, sets *total.
__device__ static inline uint64_t block_scan_u64(uint64_t x, uint64_t* s_wave, uint64_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint64_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) s_wave[wave] = inc;
  __syncthreads();
  uint64_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < CWG / 64; ++w) {
    const uint64_t v = s_wave[w];
    if (w < wave) before += v;
    all += v;
  }
  __syncthreads();  // s_wave is reused by the next call
  *total = all;
  return before + inc - x;
}

__device__ static inline void load_group(const uint8_t* t, uint64_t n, uint64_t g, uint32_t w[32]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    u32x4 v = {0, 0, 0, 0};
    if (g * 32 + 4 * q < n) v = __builtin_nontemporal_load((const u32x4*)(t + g * 128 + 16 * q));
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
}

// ---- analysis ---------------------------------------------------------------------------------

__global__ __launch_bounds__(CWG) void k_tpz_analyze(const uint8_t* __restrict__ raw,
                                                     uint64_t len, uint64_t tile,
                                                     tpz_plane* __restrict__ meta,
                                                     uint8_t* __restrict__ hlen,
                                                     uint32_t* __restrict__ hwords,
                                                     uint32_t* __restrict__ csize) {
  __shared__ uint32_t hist[4][256];
  __shared__ uint8_t rank[4][256];
  __shared__ uint16_t rc[4][256];  // rank | HUF bits << 8 per byte value (one lookup)
  __shared__ tpz_plane hdr[4];
  __shared__ uint8_t s_len[4][16];
  __shared__ uint32_t s_cnt[4][16];
  __shared__ tpz_huf_work s_work[4];
  __shared__ uint32_t s_hits[CWG / 64][20];  // 16 hit counters + 4 HUF word sums
  __shared__ uint32_t s_size[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t tbase = (uint64_t)blockIdx.x * tile;
  const uint64_t tlen = cmin64(tile, len - tbase);
  const uint8_t* t = raw + tbase;
  const uint64_t n = tlen / 4, ngroups = tpz_ngroups(tlen);

  for (int i = tid; i < 4 * 256; i += CWG) (&hist[0][0])[i] = 0;
  __syncthreads();
  const uint64_t S = n < TPZ_SAMPLE ? n : TPZ_SAMPLE;
  const uint64_t step = n / S;
  for (uint64_t j = tid; j < S; j += CWG) {
    const uint32_t w = *(const uint32_t*)(t + 4 * (j * step));
    atomicAdd(&hist[0][w & 0xff], 1u);
    atomicAdd(&hist[1][(w >> 8) & 0xff], 1u);
    atomicAdd(&hist[2][(w >> 16) & 0xff], 1u);
    atomicAdd(&hist[3][w >> 24], 1u);
  }
  __syncthreads();

  {  // wave p selects the dictionary of plane p
    const int p = wave;
    uint32_t c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = hist[p][4 * lane + i];
    int m = 0;
    for (; m < TPZ_MAXDICT; ++m) {
      uint32_t key = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t v = 4 * lane + i;
        const uint32_t kk = c[i] ? (c[i] << 8) | (255u - v) : 0u;
        key = kk > key ? kk : key;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t y = __shfl_xor(key, o, 64);
        key = y > key ? y : key;
      }
      if (key == 0) break;
      const uint32_t v = 255u - (key & 255u);
      if ((int)(v >> 2) == lane) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if ((int)(v & 3) == i) c[i] = 0;
      }
      if (lane == 0) hdr[p].dict[m] = (uint8_t)v;
    }
    if (lane == 0) hdr[p].m = (uint8_t)m;
    // rank table of plane p
    for (int v = lane; v < 256; v += 64) rank[p][v] = 15;
    if (lane < 16) s_len[p][lane] = 0;
  }
  __syncthreads();
  if (tid < 4) {  // rank table + Huffman code lengths of plane tid
    const int p = tid, m = hdr[p].m;
    for (int r = 0; r < m; ++r) rank[p][hdr[p].dict[r]] = (uint8_t)r;
    tpz_huf_counts(hist[p], hdr[p].dict, m, (uint32_t)S, s_cnt[p]);
    tpz_huf_lengths(s_cnt[p], m + 1, s_len[p], &s_work[p]);
  }
  __syncthreads();
  for (int i = tid; i < 4 * 256; i += CWG) {
    const int p = i >> 8;
    const uint32_t r = rank[p][i & 255], m = hdr[p].m;
    rc[p][i & 255] = (uint16_t)(r | (uint32_t)(r < m ? s_len[p][r] : s_len[p][m] + 8) << 8);
  }
  __syncthreads();

  // exact hits per plane for thresholds rank < 1, 3, 7, 15; HUF bits of substream tid
  uint32_t hits[4][4], bits[4] = {0, 0, 0, 0};
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) hits[p][q] = 0;
  for (uint64_t g = tid; g < ngroups; g += CWG) {
    uint32_t w[32];
    load_group(t, n, g, w);
    const uint32_t valid = (uint32_t)cmin64(32, n - g * 32);
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if ((uint32_t)j < valid) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const uint32_t v = (w[j] >> (8 * p)) & 0xff;
          const uint32_t e = rc[p][v], r = e & 0xff;
          hits[p][0] += r < 1;
          hits[p][1] += r < 3;
          hits[p][2] += r < 7;
          hits[p][3] += r < 15;
          bits[p] += e >> 8;
        }
      }
    }
  }
  uint32_t words[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    words[p] = (bits[p] + 31) >> 5;
    hwords[((uint64_t)blockIdx.x * 4 + p) * CWG + tid] = words[p];
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t v = hits[p][q];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0) s_hits[wave][4 * p + q] = v;
    }
    uint32_t v = words[p];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_hits[wave][16 + p] = v;
  }
  __syncthreads();
  if (tid < 4) {
    const int p = tid;
    uint64_t h[4], hw = 0;
    for (int q = 0; q < 4; ++q) {
      h[q] = 0;
      for (int w = 0; w < CWG / 64; ++w) h[q] += s_hits[w][4 * p + q];
    }
    for (int w = 0; w < CWG / 64; ++w) hw += s_hits[w][16 + p];
    const uint64_t huf = (hdr[p].m >= 1 && h[0] != n) ? hw : ~0ull;
    uint64_t nesc = 0;
    const int k = tpz_choose(n, ngroups, hdr[p].m, h, huf, &nesc);
    tpz_plane out;
    out.k = (uint8_t)k;
    out.pad[0] = out.pad[1] = 0;
    out.nesc = (uint32_t)nesc;
    const int used = tpz_used(k, hdr[p].m);
    out.m = (uint8_t)used;
    for (int r = 0; r < 16; ++r) out.dict[r] = r < used ? hdr[p].dict[r] : 0;
    meta[(uint64_t)blockIdx.x * 4 + p] = out;
    for (int i = 0; i < 16; ++i)
      hlen[((uint64_t)blockIdx.x * 4 + p) * 16 + i] = k == TPZ_HUF ? s_len[p][i] : 0;
    s_size[p] = (uint32_t)tpz_plane_bytes(k, ngroups, nesc);
  }
  __syncthreads();
  if (tid == 0) csize[blockIdx.x] = TPZ_HDR + s_size[0] + s_size[1] + s_size[2] + s_size[3];
}

// ---- encode -------------------------------------------------------------------------------------

template <int K>
__device__ static inline uint32_t encode_codes(const uint32_t w[32], int p, const uint8_t* rk,
                                               uint32_t valid, uint8_t* dst) {
  constexpr uint32_t E = (1u << K) - 1;
  uint32_t cw[K + 1];
#pragma unroll
  for (int i = 0; i <= K; ++i) cw[i] = 0;
  uint32_t mask = 0;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    uint32_t c = 0;
    if ((uint32_t)j < valid) {
      const uint32_t r = rk[(w[j] >> (8 * p)) & 0xff];
      c = r < E ? r : E;
      mask |= (c == E ? 1u : 0u) << j;
    }
    const int bit = j * K;
    cw[bit >> 5] |= c << (bit & 31);
    if ((bit & 31) + K > 32) cw[(bit >> 5) + 1] |= c >> (32 - (bit & 31));
  }
  if (K == 4) {
    *(u32x4*)dst = u32x4{cw[0], cw[1], cw[2], cw[3]};
  } else if (K == 2) {
    *(u32x2*)dst = u32x2{cw[0], cw[1]};
  } else {
#pragma unroll
    for (int i = 0; i < K; ++i) ((uint32_t*)dst)[i] = cw[i];
  }
  return mask;
}

// Appends the HUF codes of one group's (valid) plane-p bytes to the lane's substream: LSB-first
// bit buffer, a full u32 word is stored as soon as it exists (<= 19 bits per symbol).
// `tab[v]` = the complete bits of byte value v (its code, or the escape code followed by v)
// | their count << 24: one LDS lookup per symbol.
__device__ static inline void huf_encode_group(const uint32_t w[32], int p, uint32_t valid,
                                               const uint32_t* tab, uint64_t& acc, int& nb,
                                               uint32_t* __restrict__ stream, uint64_t& wp) {
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    if ((uint32_t)j < valid) {
      const uint32_t e = tab[(w[j] >> (8 * p)) & 0xff];
      acc |= (uint64_t)(e & 0xffffffu) << nb;
      nb += (int)(e >> 24);
      if (nb >= 32) {
        stream[wp++] = (uint32_t)acc;
        acc >>= 32;
        nb -= 32;
      }
    }
  }
}

struct PlaneGeo {
  uint64_t sec, esc;  // byte offsets in the blob
  int k;
  uint32_t nesc;
};

__device__ static inline void plane_geometry(const tpz_plane* h, uint64_t ngroups, PlaneGeo g[4],
                                             uint64_t* blob_bytes) {
  uint64_t off = TPZ_HDR;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    g[p].k = h[p].k;
    g[p].nesc = h[p].nesc;
    g[p].sec = off;
    g[p].esc = (g[p].k >= 1 && g[p].k <= 4) ? off + tpz_align16(ngroups * 4 * (uint64_t)g[p].k)
                                            : off;
    off += tpz_plane_bytes(g[p].k, ngroups, h[p].nesc);
  }
  *blob_bytes = off;
}

__global__ __launch_bounds__(CWG) void k_tpz_encode(const uint8_t* __restrict__ raw, uint64_t len,
                                                    uint64_t tile,
                                                    const tpz_plane* __restrict__ meta,
                                                    const uint8_t* __restrict__ hlen,
                                                    const uint32_t* __restrict__ hwords,
                                                    const uint32_t* __restrict__ csize,
                                                    uint32_t* __restrict__ csize_host,
                                                    uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) tpz_plane hdr[4];
  __shared__ uint8_t rank[4][256];
  __shared__ uint8_t s_clen[4][16];
  __shared__ uint16_t s_code[4][16];
  __shared__ uint32_t s_henc[4][256];  // HUF: bits | count << 24 per byte value
  __shared__ uint64_t s_wave[CWG / 64];
  const int tid = threadIdx.x;
  const uint64_t tbase = (uint64_t)blockIdx.x * tile;
  const uint64_t tlen = cmin64(tile, len - tbase);
  const uint8_t* t = raw + tbase;
  const uint64_t n = tlen / 4, ngroups = tpz_ngroups(tlen);

  // the host learns the blob sizes here, without a copy (engine.hip meta_view)
  if (tid == 0 && csize_host) tpi_sys_store(&csize_host[blockIdx.x], csize[blockIdx.x]);
  uint64_t part = 0;
  for (uint64_t i = tid; i < blockIdx.x; i += CWG) part += csize[i];
  uint64_t obase;
  block_scan_u64(part, s_wave, &obase);
  uint8_t* blob = out + obase;

  if (tid < 4) hdr[tid] = meta[(uint64_t)blockIdx.x * 4 + tid];
  if (tid < 64) s_clen[tid >> 4][tid & 15] = hlen[(uint64_t)blockIdx.x * 64 + tid];
  __syncthreads();
  if (tid < 4 && hdr[tid].k == TPZ_HUF) tpz_huf_codes(s_clen[tid], hdr[tid].m + 1, s_code[tid]);
  for (int i = tid; i < 4 * 256; i += CWG) {
    const int p = i >> 8, v = i & 255;
    uint8_t r = 15;
    for (int q = 0; q < hdr[p].m; ++q)
      if (hdr[p].dict[q] == v) r = (uint8_t)q;
    rank[p][v] = (hdr[p].k == TPZ_RAW || hdr[p].k == 0) ? 15 : r;
  }
  if (tid < TPZ_HDR / 16) ((u32x4*)blob)[tid] = ((const u32x4*)&hdr[0])[tid];
  __syncthreads();
  for (int i = tid; i < 4 * 256; i += CWG) {
    const int p = i >> 8, v = i & 255;
    if (hdr[p].k != TPZ_HUF) continue;
    const uint32_t m = hdr[p].m, r = rank[p][v], c = r < m ? r : m;
    uint32_t bits = s_code[p][c], l = s_clen[p][c];
    if (c == m) {
      bits |= (uint32_t)v << l;
      l += 8;
    }
    s_henc[p][v] = bits | (l << 24);
  }
  __syncthreads();
  PlaneGeo geo[4];
  uint64_t blob_bytes;
  plane_geometry(hdr, ngroups, geo, &blob_bytes);

  // HUF planes: code lengths, substream end offsets (lane s starts where the scan of the
  // analyzed sizes puts it), zeroed alignment padding; then one bit cursor per lane and plane
  const uint64_t S = tpz_huf_streams(ngroups);
  uint64_t hacc[4] = {0, 0, 0, 0}, hwp[4] = {0, 0, 0, 0};
  int hnb[4] = {0, 0, 0, 0};
  uint32_t* hstr[4] = {nullptr, nullptr, nullptr, nullptr};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (geo[p].k != TPZ_HUF) continue;  // uniform: the header lives in LDS
    uint8_t* sec = blob + geo[p].sec;
    uint32_t* ends = (uint32_t*)(sec + 16);
    hstr[p] = (uint32_t*)(sec + 16 + tpz_align16(4 * S));
    const uint32_t mine = hwords[((uint64_t)blockIdx.x * 4 + p) * CWG + tid];
    uint64_t tot;
    hwp[p] = block_scan_u64(mine, s_wave, &tot);
    if (tid < 16) sec[tid] = s_clen[p][tid];
    if (tid < S) ends[tid] = (uint32_t)(hwp[p] + mine);
    for (uint64_t i = S + tid; i < tpz_align16(4 * S) / 4; i += CWG) ends[i] = 0;
    for (uint64_t i = geo[p].nesc + tid; i < tpz_align16(4 * (uint64_t)geo[p].nesc) / 4; i += CWG)
      hstr[p][i] = 0;
  }

  uint64_t run[4] = {0, 0, 0, 0};
  for (uint64_t base = 0; base < ngroups; base += CWG) {
    const uint64_t g = base + tid;
    uint32_t w[32];
    uint32_t mask[4] = {0, 0, 0, 0};
    const bool live = g < ngroups;
    if (live) {
      load_group(t, n, g, w);
      const uint32_t valid = (uint32_t)cmin64(32, n - g * 32);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint8_t* sec = blob + geo[p].sec;
        switch (geo[p].k) {
          case TPZ_RAW: {
            u32x4 a, b;
            uint32_t v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
              v[q] = ((w[4 * q] >> (8 * p)) & 0xff) | (((w[4 * q + 1] >> (8 * p)) & 0xff) << 8) |
                     (((w[4 * q + 2] >> (8 * p)) & 0xff) << 16) |
                     (((w[4 * q + 3] >> (8 * p)) & 0xff) << 24);
            a = u32x4{v[0], v[1], v[2], v[3]};
            b = u32x4{v[4], v[5], v[6], v[7]};
            __builtin_nontemporal_store(a, (u32x4*)(sec + g * 32));
            __builtin_nontemporal_store(b, (u32x4*)(sec + g * 32 + 16));
            break;
          }
          case 1: mask[p] = encode_codes<1>(w, p, rank[p], valid, sec + g * 4); break;
          case 2: mask[p] = encode_codes<2>(w, p, rank[p], valid, sec + g * 8); break;
          case 3: mask[p] = encode_codes<3>(w, p, rank[p], valid, sec + g * 12); break;
          case 4: mask[p] = encode_codes<4>(w, p, rank[p], valid, sec + g * 16); break;
          case TPZ_HUF:
            huf_encode_group(w, p, valid, s_henc[p], hacc[p], hnb[p], hstr[p], hwp[p]);
            break;
          default: break;  // CONST: nothing stored
        }
      }
    }
    const uint64_t packed = (uint64_t)__popc(mask[0]) | ((uint64_t)__popc(mask[1]) << 16) |
                            ((uint64_t)__popc(mask[2]) << 32) | ((uint64_t)__popc(mask[3]) << 48);
    uint64_t tot;
    const uint64_t pre = block_scan_u64(packed, s_wave, &tot);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      uint32_t m = mask[p];
      if (m) {
        uint8_t* esc = blob + geo[p].esc + run[p] + ((pre >> (16 * p)) & 0xffff);
        int e = 0;
        while (m) {
          const int j = __ffs(m) - 1;
          m &= m - 1;
          esc[e++] = (uint8_t)((w[j] >> (8 * p)) & 0xff);
        }
      }
      run[p] += (tot >> (16 * p)) & 0xffff;
    }
  }
#pragma unroll
  for (int p = 0; p < 4; ++p)  // the last, partial word of each HUF substream
    if (geo[p].k == TPZ_HUF && hnb[p] > 0) hstr[p][hwp[p]++] = (uint32_t)hacc[p];
  // zero the alignment padding of every section (keeps blobs deterministic)
  for (int p = 0; p < 4; ++p) {
    const int k = geo[p].k;
    if (k >= 1 && k <= 4) {
      const uint64_t cend = geo[p].sec + ngroups * 4 * (uint64_t)k;
      for (uint64_t i = cend + tid; i < geo[p].esc; i += CWG) blob[i] = 0;
      const uint64_t eend = geo[p].esc + geo[p].nesc;
      const uint64_t send = geo[p].esc + tpz_align16(geo[p].nesc);
      for (uint64_t i = eend + tid; i < send; i += CWG) blob[i] = 0;
    }
  }
}

// ---- decode -------------------------------------------------------------------------------------

template <int K>
__device__ static inline uint32_t decode_codes(const uint8_t* src, const uint8_t* dict, int p,
                                               uint32_t w[32]) {
  constexpr uint32_t E = (1u << K) - 1;
  uint32_t cw[K + 1];
  if (K == 4) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4*)src);
    cw[0] = v.x; cw[1] = v.y; cw[2] = v.z; cw[3] = v.w;
  } else if (K == 2) {
    const u32x2 v = *(const u32x2*)src;
    cw[0] = v.x; cw[1] = v.y;
  } else {
#pragma unroll
    for (int i = 0; i < K; ++i) cw[i] = ((const uint32_t*)src)[i];
  }
  cw[K] = 0;
  uint32_t mask = 0;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int bit = j * K;
    uint32_t c = cw[bit >> 5] >> (bit & 31);
    if ((bit & 31) + K > 32) c |= cw[(bit >> 5) + 1] << (32 - (bit & 31));
    c &= E;
    mask |= (c == E ? 1u : 0u) << j;
    const uint32_t v = dict[c < E ? c : 0];
    w[j] |= (c < E ? v : 0u) << (8 * p);  // escapes are filled in after the scan
  }
  return mask;
}

// Decodes one group's (valid) plane-p bytes from the lane's HUF substream into w[].  Words past
// the substream's end read as zero (a corrupt blob decodes garbage; the tile CRC reports it).
__device__ static inline void huf_decode_group(const uint32_t* __restrict__ stream,
                                               const uint16_t* lut, const uint8_t* dict,
                                               uint32_t m, int p, uint32_t valid,
                                               uint64_t& acc, int& nb, uint32_t& ptr,
                                               uint32_t end, uint32_t& nxt, uint32_t w[32]) {
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    if ((uint32_t)j < valid) {
      if (nb < 32) {  // consume the word loaded one refill ago, start loading the next one
        acc |= (uint64_t)nxt << nb;
        nb += 32;
        nxt = ptr < end ? stream[ptr] : 0u;
        ++ptr;
      }
      const uint32_t e = lut[acc & (TPZ_HUF_LUT - 1)];
      const uint32_t c = e & 0xff, l = e >> 8;
      acc >>= l;
      nb -= (int)l;
      uint32_t v;
      if (c == m) {
        v = (uint32_t)acc & 0xff;
        acc >>= 8;
        nb -= 8;
      } else {
        v = dict[c & 15];
      }
      w[j] |= v << (8 * p);
    }
  }
}

// coff[i] = offset of tile i's blob relative to `comp` + comp_base; coff has ntiles+1 entries.
__global__ __launch_bounds__(CWG) void k_tpz_decode(const uint8_t* __restrict__ comp,
                                                    const uint64_t* __restrict__ coff,
                                                    uint64_t comp_base, uint64_t len,
                                                    uint64_t tile, uint8_t* __restrict__ raw) {
  __shared__ tpz_plane hdr[4];
  __shared__ uint8_t dict[4][16];
  __shared__ uint8_t s_len[4][16];
  __shared__ uint16_t s_rev[4][16];
  __shared__ uint16_t lut[4][TPZ_HUF_LUT];  // HUF: low 11 stream bits -> symbol | length << 8
  __shared__ uint64_t s_wave[CWG / 64];
  __shared__ int s_ok;
  const int tid = threadIdx.x;
  const uint64_t tbase = (uint64_t)blockIdx.x * tile;
  const uint64_t tlen = cmin64(tile, len - tbase);
  uint8_t* t = raw + tbase;
  const uint64_t n = tlen / 4, ngroups = tpz_ngroups(tlen);
  // coff may be the host's pinned offset array itself (engine.hip meta_view)
  const uint64_t b0 = tpi_sys_load(&coff[blockIdx.x]) - comp_base;
  const uint64_t b1 = tpi_sys_load(&coff[blockIdx.x + 1]) - comp_base;
  const uint8_t* blob = comp + b0;
  const uint64_t avail = b1 - b0;

  if (tid == 0) {
    int ok = avail >= TPZ_HDR;
    if (ok) {
      for (int p = 0; p < 4; ++p) hdr[p] = ((const tpz_plane*)blob)[p];
      uint64_t off = TPZ_HDR;
      for (int p = 0; p < 4 && ok; ++p) {
        const int k = hdr[p].k;
        if (!(k == TPZ_RAW || k == TPZ_HUF || k <= 4)) ok = 0;
        if (hdr[p].nesc > (k == TPZ_HUF ? 8 * n + ngroups : n)) ok = 0;
        if (k != TPZ_RAW && (hdr[p].m < 1 || hdr[p].m > TPZ_MAXDICT)) ok = 0;
        if (!ok) break;
        const uint64_t bytes = tpz_plane_bytes(k, ngroups, hdr[p].nesc);
        if (off + bytes > avail) ok = 0;
        if (ok && k == TPZ_HUF) {  // code lengths must form a complete prefix code
          for (int s = 0; s < 16; ++s) s_len[p][s] = blob[off + s];
          for (int s = hdr[p].m + 1; s < 16; ++s)
            if (s_len[p][s]) ok = 0;
          if (ok && !tpz_huf_codes(s_len[p], hdr[p].m + 1, s_rev[p])) ok = 0;
        }
        off += bytes;
      }
    }
    if (!ok)  // corrupt blob: decode as zeros; the tile CRC check reports it
      for (int p = 0; p < 4; ++p) {
        hdr[p].k = 0;
        hdr[p].m = 1;
        hdr[p].nesc = 0;
        for (int r = 0; r < 16; ++r) hdr[p].dict[r] = 0;
      }
    s_ok = ok;
  }
  __syncthreads();
  if (tid < 64) dict[tid >> 4][tid & 15] = hdr[tid >> 4].dict[tid & 15];
  for (int p = 0; p < 4; ++p) {  // decode tables of the HUF planes (uniform branch)
    if (hdr[p].k != TPZ_HUF) continue;
    const int m = hdr[p].m;
    for (int i = tid; i < TPZ_HUF_LUT; i += CWG) {
      uint16_t e = 0;
      for (int s = 0; s <= m; ++s) {
        const uint32_t l = s_len[p][s];
        if ((i & ((1u << l) - 1)) == s_rev[p][s]) e = (uint16_t)(s | (l << 8));
      }
      lut[p][i] = e;
    }
  }
  __syncthreads();
  PlaneGeo geo[4];
  uint64_t blob_bytes;
  plane_geometry(hdr, ngroups, geo, &blob_bytes);

  // HUF cursors: lane s reads substream s = [end[s-1], end[s]) of each HUF plane
  const uint64_t S = tpz_huf_streams(ngroups);
  uint64_t hacc[4] = {0, 0, 0, 0};
  int hnb[4] = {0, 0, 0, 0};
  uint32_t hptr[4] = {0, 0, 0, 0}, hend[4] = {0, 0, 0, 0}, hnxt[4] = {0, 0, 0, 0};
  const uint32_t* hstr[4] = {nullptr, nullptr, nullptr, nullptr};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (geo[p].k != TPZ_HUF) continue;
    const uint8_t* sec = blob + geo[p].sec;
    hstr[p] = (const uint32_t*)(sec + 16 + tpz_align16(4 * S));
    if (tid < S) {
      const uint32_t* ends = (const uint32_t*)(sec + 16);
      const uint32_t e = ends[tid], s0 = tid ? ends[tid - 1] : 0u;
      if (s0 <= e && e <= geo[p].nesc) {
        hptr[p] = s0;
        hend[p] = e;
      }
    }
    hnxt[p] = hptr[p] < hend[p] ? hstr[p][hptr[p]] : 0u;  // software-pipelined refills
    ++hptr[p];
  }

  uint64_t run[4] = {0, 0, 0, 0};
  for (uint64_t base = 0; base < ngroups; base += CWG) {
    const uint64_t g = base + tid;
    uint32_t w[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) w[j] = 0;
    uint32_t mask[4] = {0, 0, 0, 0};
    const bool live = g < ngroups;
    if (live) {
      const uint32_t valid = (uint32_t)cmin64(32, n - g * 32);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint8_t* sec = blob + geo[p].sec;
        switch (geo[p].k) {
          case TPZ_RAW: {
            const u32x4 a = __builtin_nontemporal_load((const u32x4*)(sec + g * 32));
            const u32x4 b = __builtin_nontemporal_load((const u32x4*)(sec + g * 32 + 16));
            const uint32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int j = 0; j < 32; ++j) w[j] |= ((v[j >> 2] >> (8 * (j & 3))) & 0xff) << (8 * p);
            break;
          }
          case 0: {
            const uint32_t c = (uint32_t)dict[p][0] << (8 * p);
#pragma unroll
            for (int j = 0; j < 32; ++j) w[j] |= c;
            break;
          }
          case 1: mask[p] = decode_codes<1>(sec + g * 4, dict[p], p, w); break;
          case 2: mask[p] = decode_codes<2>(sec + g * 8, dict[p], p, w); break;
          case 3: mask[p] = decode_codes<3>(sec + g * 12, dict[p], p, w); break;
          case 4: mask[p] = decode_codes<4>(sec + g * 16, dict[p], p, w); break;
          case TPZ_HUF:
            huf_decode_group(hstr[p], lut[p], dict[p], hdr[p].m, p, valid, hacc[p], hnb[p],
                             hptr[p], hend[p], hnxt[p], w);
            break;
          default: break;
        }
      }
      if (valid < 32) {
        const uint32_t keep = (1u << valid) - 1;
#pragma unroll
        for (int p = 0; p < 4; ++p) mask[p] &= keep;
      }
    }
    const uint64_t packed = (uint64_t)__popc(mask[0]) | ((uint64_t)__popc(mask[1]) << 16) |
                            ((uint64_t)__popc(mask[2]) << 32) | ((uint64_t)__popc(mask[3]) << 48);
    uint64_t tot;
    const uint64_t pre = block_scan_u64(packed, s_wave, &tot);
    if (live) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint32_t m = mask[p];
        uint64_t e = run[p] + ((pre >> (16 * p)) & 0xffff);
        const uint8_t* esc = blob + geo[p].esc;
        while (m) {
          const int j = __ffs(m) - 1;
          m &= m - 1;
          const uint32_t v = e < geo[p].nesc ? esc[e] : 0u;
          ++e;
#pragma unroll
          for (int jj = 0; jj < 32; ++jj)  // register-resident w[]: select, no dynamic index
            if (jj == j) w[jj] |= v << (8 * p);
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (g * 32 + 4 * q < n)
          __builtin_nontemporal_store(u32x4{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]},
                                      (u32x4*)(t + g * 128 + 16 * q));
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) run[p] += (tot >> (16 * p)) & 0xffff;
  }
  (void)s_ok;
}

// ---- launchers ------------------------------------------------------------------------------------

extern "C" hipError_t tpi_launch_tpz_encode(const void* raw, uint64_t len, uint64_t tile,
                                            void* meta, uint32_t* csize, uint32_t* csize_host,
                                            void* out, hipStream_t stream) {
  if (len == 0) return hipSuccess;
  const unsigned ntiles = (unsigned)((len + tile - 1) / tile);
  // meta (tpz_meta_bytes(ntiles)): plane headers | HUF code lengths | HUF substream words
  uint8_t* mb = (uint8_t*)meta;
  tpz_plane* planes = (tpz_plane*)mb;
  uint8_t* hlen = mb + (uint64_t)ntiles * TPZ_HDR;
  uint32_t* hwords = (uint32_t*)(mb + (uint64_t)ntiles * (TPZ_HDR + 64));
  hipLaunchKernelGGL(k_tpz_analyze, dim3(ntiles), dim3(CWG), 0, stream, (const uint8_t*)raw, len,
                     tile, planes, hlen, hwords, csize);
  hipLaunchKernelGGL(k_tpz_encode, dim3(ntiles), dim3(CWG), 0, stream, (const uint8_t*)raw, len,
                     tile, (const tpz_plane*)planes, (const uint8_t*)hlen,
                     (const uint32_t*)hwords, (const uint32_t*)csize, csize_host,
                     (uint8_t*)out);
  return hipGetLastError();
}

extern "C" hipError_t tpi_launch_tpz_decode(const void* comp, const uint64_t* coff,
                                            uint64_t comp_base, uint64_t len, uint64_t tile,
                                            void* raw, hipStream_t stream) {
  if (len == 0) return hipSuccess;
  const unsigned ntiles = (unsigned)((len + tile - 1) / tile);
  hipLaunchKernelGGL(k_tpz_decode, dim3(ntiles), dim3(CWG), 0, stream, (const uint8_t*)comp, coff,
                     comp_base, len, tile, (uint8_t*)raw);
  return hipGetLastError();
}
