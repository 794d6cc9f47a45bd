// TPZ1: lossless byte-plane dictionary codec for checkpoint tiles (host reference + format).
//
// Checkpoint PCIe spill is link-bound (~56 GB/s per MI355X), so bytes removed before the D2H
// are throughput gained.  Model state is floating point: the byte holding sign + high exponent
// bits of every bf16/fp32 element takes only a handful of values, while mantissa bytes are
// noise.  A tile (the CRC tile of the packed stream, a multiple of 16 bytes) is therefore seen
// as 4 byte planes (plane p = bytes at offsets 4i+p) and each plane is coded independently:
//
//   RAW      (k=8)  the plane bytes as they are
//   CONST    (k=0)  every byte equals dict[0]
//   DICT(k)  k=1..4: k-bit codes; code c < E=2^k-1 -> dict[c]; code E -> next escape byte
//
// The dictionary is the (up to 15) most frequent byte values of a fixed sample of the tile
// (count desc, value asc); k is then chosen from EXACT per-tile hit counts to minimise the
// plane's coded size.  Everything is deterministic, so the GPU encoder
// (csrc/hip/codec.hip) and this host reference produce byte-identical blobs.
//
// Tile blob (all sections 16-byte aligned):
//   tpz_plane hdr[4]                                  96 bytes
//   for p in 0..3:  codes (DICT: ngroups*4*k bytes, RAW: ngroups*32 bytes, CONST: none)
//                   escapes (nesc bytes, DICT only)
// A group is 32 consecutive plane bytes (= 128 tile bytes); code j of a group sits at bit
// j*k of the group's k little-endian u32 words.  Positions past the tile end are padding
// (code 0 / byte 0, never escapes).
#pragma once
#include <stdint.h>
#include <string.h>

#define TPZ_HDR 96
#define TPZ_SAMPLE 4096  // sampled u32 words per tile for the dictionary
#define TPZ_MAXDICT 15
#define TPZ_RAW 8

struct tpz_plane {
  uint8_t k;      // 0, 1..4, or TPZ_RAW
  uint8_t m;      // dictionary entries in use
  uint8_t pad[2];
  uint32_t nesc;  // escape bytes (DICT)
  uint8_t dict[16];
};
static_assert(sizeof(tpz_plane) == 24, "tpz_plane layout");

#if defined(__HIPCC__)
#define TPZ_HD __host__ __device__
#else
#define TPZ_HD
#endif

#ifdef __cplusplus
TPZ_HD static inline uint64_t tpz_align16(uint64_t x) { return (x + 15) & ~15ull; }
TPZ_HD static inline uint64_t tpz_ngroups(uint64_t len) { return (len / 4 + 31) / 32; }

// Coded size of one plane section (codes + escapes).
TPZ_HD static inline uint64_t tpz_plane_bytes(int k, uint64_t ngroups, uint64_t nesc) {
  if (k == TPZ_RAW) return ngroups * 32;
  if (k == 0) return 0;
  return tpz_align16(ngroups * 4 * (uint64_t)k) + tpz_align16(nesc);
}

// Worst-case blob size of a tile of `len` bytes.
TPZ_HD static inline uint64_t tpz_bound(uint64_t len) { return TPZ_HDR + 4 * tpz_ngroups(len) * 32; }

// Given exact hit counts hits[t] = #bytes with rank < {1,3,7,15}[t], pick the cheapest mode.
TPZ_HD static inline int tpz_choose(uint64_t n, uint64_t ngroups, int m, const uint64_t hits[4],
                             uint64_t* nesc_out) {
  int best = TPZ_RAW;
  uint64_t best_cost = ngroups * 32, best_nesc = 0;
  if (m >= 1 && hits[0] == n) {
    best = 0;
    best_cost = 0;
  } else {
    for (int k = 1; k <= 4 && m >= 1; ++k) {
      const uint64_t nesc = n - hits[k - 1];
      const uint64_t cost = tpz_plane_bytes(k, ngroups, nesc);
      if (cost < best_cost) {
        best = k;
        best_cost = cost;
        best_nesc = nesc;
      }
    }
  }
  *nesc_out = best == TPZ_RAW || best == 0 ? 0 : best_nesc;
  return best;
}

// Top-m byte values of a 256-bin histogram: count desc, value asc, count > 0.
static inline int tpz_topk(const uint32_t* hist, uint8_t* dict) {
  uint8_t taken[256];
  memset(taken, 0, sizeof(taken));
  int m = 0;
  for (; m < TPZ_MAXDICT; ++m) {
    int bv = -1;
    uint32_t bc = 0;
    for (int v = 0; v < 256; ++v)
      if (!taken[v] && hist[v] > bc) {
        bc = hist[v];
        bv = v;
      }
    if (bv < 0) break;
    taken[bv] = 1;
    dict[m] = (uint8_t)bv;
  }
  return m;
}

static inline uint32_t tpz_word(const uint8_t* t, uint64_t len, uint64_t w) {
  uint32_t x = 0;
  if (4 * w + 4 <= len) memcpy(&x, t + 4 * w, 4);
  return x;
}

// Pass 1 (= k_tpz_analyze): dictionaries, exact hit counts and the mode of every plane.
// Fills hdr[4] and returns the blob size.
static inline uint64_t tpz_analyze_tile(const uint8_t* t, uint64_t len, tpz_plane hdr[4]) {
  const uint64_t n = len / 4, ngroups = tpz_ngroups(len);
  memset(hdr, 0, 4 * sizeof(tpz_plane));
  uint8_t rank[4][256];
  {
    uint32_t hist[4][256];
    memset(hist, 0, sizeof(hist));
    const uint64_t S = n < TPZ_SAMPLE ? n : TPZ_SAMPLE;
    const uint64_t step = n / S;
    for (uint64_t j = 0; j < S; ++j) {
      const uint32_t w = tpz_word(t, len, j * step);
      for (int p = 0; p < 4; ++p) hist[p][(w >> (8 * p)) & 0xff]++;
    }
    for (int p = 0; p < 4; ++p) {
      hdr[p].m = (uint8_t)tpz_topk(hist[p], hdr[p].dict);
      memset(rank[p], 15, 256);
      for (int r = 0; r < hdr[p].m; ++r) rank[p][hdr[p].dict[r]] = (uint8_t)r;
    }
  }
  // hits[p][r] = bytes of plane p with rank r (r = 15: not in the dictionary)
  uint64_t cnt[4][16];
  memset(cnt, 0, sizeof(cnt));
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t w;
    memcpy(&w, t + 4 * i, 4);
    cnt[0][rank[0][w & 0xff]]++;
    cnt[1][rank[1][(w >> 8) & 0xff]]++;
    cnt[2][rank[2][(w >> 16) & 0xff]]++;
    cnt[3][rank[3][w >> 24]]++;
  }
  uint64_t size = TPZ_HDR;
  for (int p = 0; p < 4; ++p) {
    uint64_t hits[4] = {0, 0, 0, 0};
    static const int thr[4] = {1, 3, 7, 15};
    for (int q = 0; q < 4; ++q)
      for (int r = 0; r < thr[q]; ++r) hits[q] += cnt[p][r];
    uint64_t nesc = 0;
    const int k = tpz_choose(n, ngroups, hdr[p].m, hits, &nesc);
    hdr[p].k = (uint8_t)k;
    hdr[p].nesc = (uint32_t)nesc;
    if (k == TPZ_RAW) {
      hdr[p].m = 0;
      memset(hdr[p].dict, 0, 16);
    } else {
      const int used = k == 0 ? 1 : ((1 << k) - 1 < hdr[p].m ? (1 << k) - 1 : hdr[p].m);
      for (int r = used; r < 16; ++r) hdr[p].dict[r] = 0;
      hdr[p].m = (uint8_t)used;
    }
    size += tpz_plane_bytes(k, ngroups, nesc);
  }
  return size;
}

// Pass 2 (= k_tpz_encode): write the blob described by `hdr` (>= its size bytes at `out`).
static inline uint64_t tpz_emit_tile(const uint8_t* t, uint64_t len, const tpz_plane hdr[4],
                                     uint8_t* out) {
  const uint64_t n = len / 4, ngroups = tpz_ngroups(len);
  memcpy(out, hdr, TPZ_HDR);
  uint64_t off = TPZ_HDR;
  for (int p = 0; p < 4; ++p) {
    const int k = hdr[p].k;
    uint8_t* sec = out + off;
    const uint64_t bytes = tpz_plane_bytes(k, ngroups, hdr[p].nesc);
    if (k == TPZ_RAW) {
      for (uint64_t i = 0; i < n; ++i) sec[i] = t[4 * i + p];
      memset(sec + n, 0, bytes - n);
    } else if (k > 0) {
      memset(sec, 0, bytes);
      uint8_t rank[256];
      memset(rank, 15, sizeof(rank));
      for (int r = 0; r < hdr[p].m; ++r) rank[hdr[p].dict[r]] = (uint8_t)r;
      const uint32_t E = (1u << k) - 1;
      uint8_t* esc = sec + tpz_align16(ngroups * 4 * (uint64_t)k);
      uint64_t ne = 0;
      for (uint64_t g = 0; g < ngroups; ++g) {
        uint64_t acc = 0;  // k <= 4: 32 codes fit in 128 bits, emitted 64 bits at a time
        int nbits = 0;
        uint8_t* dst = sec + g * 4 * k;
        for (int j = 0; j < 32; ++j) {
          const uint64_t i = g * 32 + j;
          uint32_t c = 0;
          if (i < n) {
            const uint8_t v = t[4 * i + p];
            c = rank[v];
            if (c >= E) {
              c = E;
              esc[ne++] = v;
            }
          }
          acc |= (uint64_t)c << nbits;
          nbits += k;
          if (nbits >= 64) {
            memcpy(dst, &acc, 8);
            dst += 8;
            nbits -= 64;
            acc = nbits ? (uint64_t)c >> (k - nbits) : 0;
          }
        }
        if (nbits) memcpy(dst, &acc, (size_t)(nbits + 7) / 8);
      }
    }
    off += bytes;
  }
  return off;
}

// Encode one tile (`len` % 16 == 0, len > 0) into `out` (>= tpz_bound(len) bytes).
// Returns the blob size.
static inline uint64_t tpz_encode_tile(const uint8_t* t, uint64_t len, uint8_t* out) {
  tpz_plane hdr[4];
  tpz_analyze_tile(t, len, hdr);
  return tpz_emit_tile(t, len, hdr, out);
}

// Decode a blob of `avail` bytes into `len` tile bytes.  Returns the blob size consumed, or
// 0 if the blob is malformed (bad header, truncated, escape overrun).
static inline uint64_t tpz_decode_tile(const uint8_t* blob, uint64_t avail, uint64_t len,
                                       uint8_t* t) {
  if (avail < TPZ_HDR) return 0;
  const uint64_t n = len / 4, ngroups = tpz_ngroups(len);
  tpz_plane hdr[4];
  memcpy(hdr, blob, TPZ_HDR);
  uint64_t off = TPZ_HDR;
  for (int p = 0; p < 4; ++p) {
    const int k = hdr[p].k;
    if (!(k == TPZ_RAW || (k >= 0 && k <= 4)) || hdr[p].nesc > n) return 0;
    if (k != TPZ_RAW && (hdr[p].m < 1 || hdr[p].m > TPZ_MAXDICT)) return 0;
    const uint64_t bytes = tpz_plane_bytes(k, ngroups, hdr[p].nesc);
    if (off + bytes > avail) return 0;
    const uint8_t* sec = blob + off;
    if (k == TPZ_RAW) {
      for (uint64_t i = 0; i < n; ++i) t[4 * i + p] = sec[i];
    } else if (k == 0) {
      for (uint64_t i = 0; i < n; ++i) t[4 * i + p] = hdr[p].dict[0];
    } else {
      const uint32_t E = (1u << k) - 1;
      const uint8_t* esc = sec + tpz_align16(ngroups * 4 * (uint64_t)k);
      uint64_t ne = 0;
      for (uint64_t g = 0; g < ngroups; ++g) {
        uint32_t words[5] = {0, 0, 0, 0, 0};
        memcpy(words, sec + g * 4 * k, 4 * k);
        for (int j = 0; j < 32; ++j) {
          const uint64_t i = g * 32 + j;
          if (i >= n) break;
          const int bit = j * k;
          uint32_t c = words[bit >> 5] >> (bit & 31);
          if ((bit & 31) + k > 32) c |= words[(bit >> 5) + 1] << (32 - (bit & 31));
          c &= E;
          if (c == E) {
            if (ne >= hdr[p].nesc) return 0;
            t[4 * i + p] = esc[ne++];
          } else {
            if (c >= hdr[p].m) return 0;
            t[4 * i + p] = hdr[p].dict[c];
          }
        }
      }
      if (ne != hdr[p].nesc) return 0;
    }
    off += bytes;
  }
  return off;
}
#endif
