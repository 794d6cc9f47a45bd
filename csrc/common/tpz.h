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
//   HUF      (k=9)  canonical Huffman code over the m dictionary entries + one escape symbol
//                   (symbol m, followed inline by the 8 raw bits), code lengths <= 11
//
// The dictionary is the (up to 15) most frequent byte values of a fixed sample of the tile
// (count desc, value asc); HUF code lengths come from the same sample.  The mode is then
// chosen from EXACT per-tile costs to minimise the plane's coded size.  An exponent plane of
// N(0, s) weights carries ~2.6 bits of entropy: DICT(3) spends ~3.3 bits per byte on it, HUF
// ~2.7.  Everything is deterministic, so the GPU encoder (csrc/hip/codec.hip) and this host
// reference produce byte-identical blobs.
//
// Tile blob (all sections 16-byte aligned):
//   tpz_plane hdr[4]                                  96 bytes
//   for p in 0..3:  codes (DICT: ngroups*4*k bytes, RAW: ngroups*32 bytes, CONST: none)
//                   escapes (nesc bytes, DICT only)
//                   HUF: u8 len[16] | u32 end[S] (16-aligned) | u32 words[nesc] (16-aligned)
// A group is 32 consecutive plane bytes (= 128 tile bytes); DICT code j of a group sits at bit
// j*k of the group's k little-endian u32 words.  Positions past the tile end are padding
// (code 0 / byte 0, never escapes).
//
// HUF substreams: S = min(256, ngroups); substream s codes groups s, s+256, s+512, ... (the
// groups lane s of a 256-lane workgroup visits round by round, so encoder and decoder keep one
// bit cursor per lane and no lane waits for another).  Bits are LSB-first: each code is stored
// bit-reversed so a decoder indexes a 2^11-entry table with the low 11 bits of its buffer.
// end[s] = cumulative u32 words through substream s; the plane header's nesc holds the total.
#pragma once
#include <stdint.h>
#include <string.h>

#define TPZ_HDR 96
#define TPZ_SAMPLE 4096  // sampled u32 words per tile for the dictionary
#define TPZ_MAXDICT 15
#define TPZ_RAW 8
#define TPZ_HUF 9
#define TPZ_HUF_STREAMS 256
#define TPZ_HUF_MAXLEN 11
#define TPZ_HUF_LUT (1 << TPZ_HUF_MAXLEN)
// Device scratch per tile between the analyze and encode kernels: headers, HUF code lengths
// (16 per plane), HUF words per (plane, substream).
#define TPZ_META_TILE (TPZ_HDR + 64 + 4 * TPZ_HUF_STREAMS * 4)

struct tpz_plane {
  uint8_t k;      // 0, 1..4, TPZ_RAW or TPZ_HUF
  uint8_t m;      // dictionary entries in use
  uint8_t pad[2];
  uint32_t nesc;  // escape bytes (DICT) / stream words (HUF)
  uint8_t dict[16];
};
static_assert(sizeof(tpz_plane) == 24, "tpz_plane layout");

// Workspace of tpz_huf_lengths (LDS on the device: private arrays would live in scratch).
struct tpz_huf_work {
  uint64_t w[31];
  uint32_t cnt[16];
  uint8_t parent[31];
  uint8_t alive[31];
};

#if defined(__HIPCC__)
#define TPZ_HD __host__ __device__
#else
#define TPZ_HD
#endif

#ifdef __cplusplus
TPZ_HD static inline uint64_t tpz_align16(uint64_t x) { return (x + 15) & ~15ull; }
TPZ_HD static inline uint64_t tpz_ngroups(uint64_t len) { return (len / 4 + 31) / 32; }
TPZ_HD static inline uint64_t tpz_huf_streams(uint64_t ngroups) {
  return ngroups < TPZ_HUF_STREAMS ? ngroups : TPZ_HUF_STREAMS;
}
TPZ_HD static inline uint64_t tpz_meta_bytes(uint64_t ntiles) { return ntiles * TPZ_META_TILE; }

// Coded size of one plane section.
TPZ_HD static inline uint64_t tpz_plane_bytes(int k, uint64_t ngroups, uint64_t nesc) {
  if (k == TPZ_RAW) return ngroups * 32;
  if (k == 0) return 0;
  if (k == TPZ_HUF) return 16 + tpz_align16(4 * tpz_huf_streams(ngroups)) + tpz_align16(4 * nesc);
  return tpz_align16(ngroups * 4 * (uint64_t)k) + tpz_align16(nesc);
}

// Worst-case blob size of a tile of `len` bytes.
TPZ_HD static inline uint64_t tpz_bound(uint64_t len) { return TPZ_HDR + 4 * tpz_ngroups(len) * 32; }

// Given exact hit counts hits[t] = #bytes with rank < {1,3,7,15}[t] and the HUF stream words
// (~0 when unavailable), pick the cheapest mode.  Ties keep the earlier mode.
TPZ_HD static inline int tpz_choose(uint64_t n, uint64_t ngroups, int m, const uint64_t hits[4],
                                    uint64_t huf_words, uint64_t* nesc_out) {
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
    if (m >= 1 && huf_words != ~0ull && tpz_plane_bytes(TPZ_HUF, ngroups, huf_words) < best_cost) {
      best = TPZ_HUF;
      best_nesc = huf_words;
    }
  }
  *nesc_out = best == TPZ_RAW || best == 0 ? 0 : best_nesc;
  return best;
}

// Dictionary entries a plane coded with mode k keeps out of its m candidates.
TPZ_HD static inline int tpz_used(int k, int m) {
  if (k == TPZ_RAW) return 0;
  if (k == 0) return 1;
  if (k == TPZ_HUF) return m;
  return (1 << k) - 1 < m ? (1 << k) - 1 : m;
}

// Huffman code lengths (<= TPZ_HUF_MAXLEN) of `ns` <= 16 symbols with sample counts `cnt_in`:
// repeated merge of the two lightest nodes (ties: lower node index); while the tree is too
// deep the counts are halved (kept >= 1) and the tree rebuilt.  Deterministic on host/device.
TPZ_HD static inline void tpz_huf_lengths(const uint32_t* cnt_in, int ns, uint8_t* len,
                                          tpz_huf_work* wk) {
  for (int i = 0; i < ns; ++i) wk->cnt[i] = cnt_in[i] ? cnt_in[i] : 1;
  if (ns == 1) {
    len[0] = 1;
    return;
  }
  for (;;) {
    for (int i = 0; i < ns; ++i) {
      wk->w[i] = wk->cnt[i];
      wk->alive[i] = 1;
    }
    int nn = ns;
    for (int it = 0; it < ns - 1; ++it) {
      int a = -1, b = -1;
      for (int j = 0; j < nn; ++j) {
        if (!wk->alive[j]) continue;
        if (a < 0 || wk->w[j] < wk->w[a]) {
          b = a;
          a = j;
        } else if (b < 0 || wk->w[j] < wk->w[b]) {
          b = j;
        }
      }
      wk->w[nn] = wk->w[a] + wk->w[b];
      wk->alive[nn] = 1;
      wk->alive[a] = wk->alive[b] = 0;
      wk->parent[a] = wk->parent[b] = (uint8_t)nn;
      ++nn;
    }
    const int root = nn - 1;
    int maxd = 0;
    for (int i = 0; i < ns; ++i) {
      int d = 0;
      for (int j = i; j != root; j = wk->parent[j]) ++d;
      len[i] = (uint8_t)d;
      maxd = d > maxd ? d : maxd;
    }
    if (maxd <= TPZ_HUF_MAXLEN) return;
    for (int i = 0; i < ns; ++i) wk->cnt[i] = (wk->cnt[i] >> 1) | 1;
  }
}

// Bit-reversed canonical codes (deflate order: by length, then symbol).  Returns false unless
// the lengths form a complete prefix code with every length in 1..TPZ_HUF_MAXLEN.
TPZ_HD static inline bool tpz_huf_codes(const uint8_t* len, int ns, uint16_t* rev) {
  uint32_t kraft = 0, code = 0;
  for (int i = 0; i < ns; ++i) {
    if (len[i] < 1 || len[i] > TPZ_HUF_MAXLEN) return false;
    kraft += 1u << (TPZ_HUF_MAXLEN - len[i]);
  }
  if (kraft != (1u << TPZ_HUF_MAXLEN)) return false;
  for (int bl = 1; bl <= TPZ_HUF_MAXLEN; ++bl) {
    for (int s = 0; s < ns; ++s) {
      if (len[s] != bl) continue;
      uint32_t r = 0;
      for (int b = 0; b < bl; ++b) r |= ((code >> b) & 1u) << (bl - 1 - b);
      rev[s] = (uint16_t)r;
      ++code;
    }
    code <<= 1;
  }
  return true;
}

// Huffman symbol counts of a plane from its sample histogram: the dictionary entries, then
// the escape symbol (every sampled byte outside the dictionary).
TPZ_HD static inline void tpz_huf_counts(const uint32_t* hist, const uint8_t* dict, int m,
                                         uint32_t samples, uint32_t* cnt) {
  uint32_t in = 0;
  for (int r = 0; r < m; ++r) {
    cnt[r] = hist[dict[r]];
    in += cnt[r];
  }
  cnt[m] = samples - in;
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

// Bits per byte value of a HUF plane (code length, + 8 for escaped values).
static inline void tpz_huf_costs(const tpz_plane& h, const uint8_t* len, uint8_t cost[256]) {
  for (int v = 0; v < 256; ++v) cost[v] = (uint8_t)(len[h.m] + 8);
  for (int r = 0; r < h.m; ++r) cost[h.dict[r]] = len[r];
}

// Total u32 words of the HUF substreams of plane p.
static inline uint64_t tpz_huf_total_words(const uint8_t* t, uint64_t len, int p,
                                           const uint8_t cost[256]) {
  const uint64_t n = len / 4, ngroups = tpz_ngroups(len), S = tpz_huf_streams(ngroups);
  uint64_t total = 0;
  for (uint64_t s = 0; s < S; ++s) {
    uint64_t bits = 0;
    for (uint64_t g = s; g < ngroups; g += TPZ_HUF_STREAMS) {
      const uint64_t hi = (g + 1) * 32 < n ? (g + 1) * 32 : n;
      for (uint64_t i = g * 32; i < hi; ++i) bits += cost[t[4 * i + p]];
    }
    total += (bits + 31) / 32;
  }
  return total;
}

// Pass 1 (= k_tpz_analyze): dictionaries, HUF code lengths (lens[p][0..m]), exact costs and
// the mode of every plane.  Fills hdr[4] / lens and returns the blob size.
static inline uint64_t tpz_analyze_tile(const uint8_t* t, uint64_t len, tpz_plane hdr[4],
                                        uint8_t lens[4][16]) {
  const uint64_t n = len / 4, ngroups = tpz_ngroups(len);
  memset(hdr, 0, 4 * sizeof(tpz_plane));
  memset(lens, 0, 4 * 16);
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
      uint32_t cnt[16];
      tpz_huf_work wk;
      tpz_huf_counts(hist[p], hdr[p].dict, hdr[p].m, (uint32_t)S, cnt);
      tpz_huf_lengths(cnt, hdr[p].m + 1, lens[p], &wk);
    }
  }
  // cnt[p][r] = bytes of plane p with rank r (r = 15: not in the dictionary)
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
    uint64_t huf = ~0ull;
    if (hdr[p].m >= 1 && hits[0] != n) {
      uint8_t cost[256];
      tpz_huf_costs(hdr[p], lens[p], cost);
      huf = tpz_huf_total_words(t, len, p, cost);
    }
    uint64_t nesc = 0;
    const int k = tpz_choose(n, ngroups, hdr[p].m, hits, huf, &nesc);
    hdr[p].k = (uint8_t)k;
    hdr[p].nesc = (uint32_t)nesc;
    const int used = tpz_used(k, hdr[p].m);
    for (int r = used; r < 16; ++r) hdr[p].dict[r] = 0;
    hdr[p].m = (uint8_t)used;
    if (k != TPZ_HUF) memset(lens[p], 0, 16);
    size += tpz_plane_bytes(k, ngroups, nesc);
  }
  return size;
}

// HUF section of plane p (layout in the file comment); `sec` has room for the section.
static inline void tpz_emit_huf(const uint8_t* t, uint64_t len, int p, const tpz_plane& h,
                                const uint8_t* lens, uint8_t* sec) {
  const uint64_t n = len / 4, ngroups = tpz_ngroups(len), S = tpz_huf_streams(ngroups);
  memset(sec, 0, tpz_plane_bytes(TPZ_HUF, ngroups, h.nesc));
  memcpy(sec, lens, 16);
  uint16_t rev[16];
  tpz_huf_codes(lens, h.m + 1, rev);
  uint8_t sym[256];
  memset(sym, h.m, sizeof(sym));
  for (int r = 0; r < h.m; ++r) sym[h.dict[r]] = (uint8_t)r;
  uint8_t* stream = sec + 16 + tpz_align16(4 * S);
  uint64_t wp = 0;
  for (uint64_t s = 0; s < S; ++s) {
    uint64_t acc = 0;
    int nb = 0;
    for (uint64_t g = s; g < ngroups; g += TPZ_HUF_STREAMS) {
      const uint64_t hi = (g + 1) * 32 < n ? (g + 1) * 32 : n;
      for (uint64_t i = g * 32; i < hi; ++i) {
        const uint8_t v = t[4 * i + p];
        const int c = sym[v];
        acc |= (uint64_t)rev[c] << nb;
        nb += lens[c];
        if (c == h.m) {
          acc |= (uint64_t)v << nb;
          nb += 8;
        }
        if (nb >= 32) {
          const uint32_t word = (uint32_t)acc;
          memcpy(stream + 4 * wp++, &word, 4);
          acc >>= 32;
          nb -= 32;
        }
      }
    }
    if (nb > 0) {
      const uint32_t word = (uint32_t)acc;
      memcpy(stream + 4 * wp++, &word, 4);
    }
    const uint32_t end = (uint32_t)wp;
    memcpy(sec + 16 + 4 * s, &end, 4);
  }
}

// Pass 2 (= k_tpz_encode): write the blob described by `hdr`/`lens` (>= its size bytes at
// `out`).
static inline uint64_t tpz_emit_tile(const uint8_t* t, uint64_t len, const tpz_plane hdr[4],
                                     const uint8_t lens[4][16], uint8_t* out) {
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
    } else if (k == TPZ_HUF) {
      tpz_emit_huf(t, len, p, hdr[p], lens[p], sec);
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
  uint8_t lens[4][16];
  tpz_analyze_tile(t, len, hdr, lens);
  return tpz_emit_tile(t, len, hdr, lens, out);
}

// Decode the HUF section of plane p.  Returns false if it is malformed.
static inline bool tpz_decode_huf(const uint8_t* sec, uint64_t len, int p, const tpz_plane& h,
                                  uint8_t* t) {
  const uint64_t n = len / 4, ngroups = tpz_ngroups(len), S = tpz_huf_streams(ngroups);
  const uint8_t* lens = sec;
  for (int s = h.m + 1; s < 16; ++s)
    if (lens[s]) return false;
  uint16_t rev[16];
  if (!tpz_huf_codes(lens, h.m + 1, rev)) return false;
  uint16_t lut[TPZ_HUF_LUT];
  for (int s = 0; s <= h.m; ++s)
    for (uint32_t f = 0; f < (1u << (TPZ_HUF_MAXLEN - lens[s])); ++f)
      lut[rev[s] | (f << lens[s])] = (uint16_t)(s | (lens[s] << 8));
  const uint8_t* stream = sec + 16 + tpz_align16(4 * S);
  uint64_t start = 0;
  for (uint64_t s = 0; s < S; ++s) {
    uint32_t end;
    memcpy(&end, sec + 16 + 4 * s, 4);
    if (end < start || end > h.nesc || (s + 1 == S && end != h.nesc)) return false;
    uint64_t acc = 0, ptr = start, used = 0;
    int nb = 0;
    for (uint64_t g = s; g < ngroups; g += TPZ_HUF_STREAMS) {
      const uint64_t hi = (g + 1) * 32 < n ? (g + 1) * 32 : n;
      for (uint64_t i = g * 32; i < hi; ++i) {
        if (nb < 32) {
          uint32_t word = 0;
          if (ptr < end) memcpy(&word, stream + 4 * ptr, 4);
          ++ptr;
          acc |= (uint64_t)word << nb;
          nb += 32;
        }
        const uint16_t e = lut[acc & (TPZ_HUF_LUT - 1)];
        const int c = e & 0xff, l = e >> 8;
        acc >>= l;
        nb -= l;
        used += l;
        if (c == h.m) {
          t[4 * i + p] = (uint8_t)acc;
          acc >>= 8;
          nb -= 8;
          used += 8;
        } else {
          t[4 * i + p] = h.dict[c];
        }
      }
    }
    if (used > 32 * (uint64_t)(end - start)) return false;
    start = end;
  }
  return true;
}

// Decode a blob of `avail` bytes into `len` tile bytes.  Returns the blob size consumed, or
// 0 if the blob is malformed (bad header, truncated, escape or stream overrun).
static inline uint64_t tpz_decode_tile(const uint8_t* blob, uint64_t avail, uint64_t len,
                                       uint8_t* t) {
  if (avail < TPZ_HDR) return 0;
  const uint64_t n = len / 4, ngroups = tpz_ngroups(len);
  tpz_plane hdr[4];
  memcpy(hdr, blob, TPZ_HDR);
  uint64_t off = TPZ_HDR;
  for (int p = 0; p < 4; ++p) {
    const int k = hdr[p].k;
    if (!(k == TPZ_RAW || k == TPZ_HUF || (k >= 0 && k <= 4))) return 0;
    if (hdr[p].nesc > (k == TPZ_HUF ? 8 * n + ngroups : n)) return 0;
    if (k != TPZ_RAW && (hdr[p].m < 1 || hdr[p].m > TPZ_MAXDICT)) return 0;
    const uint64_t bytes = tpz_plane_bytes(k, ngroups, hdr[p].nesc);
    if (off + bytes > avail) return 0;
    const uint8_t* sec = blob + off;
    if (k == TPZ_RAW) {
      for (uint64_t i = 0; i < n; ++i) t[4 * i + p] = sec[i];
    } else if (k == 0) {
      for (uint64_t i = 0; i < n; ++i) t[4 * i + p] = hdr[p].dict[0];
    } else if (k == TPZ_HUF) {
      if (!tpz_decode_huf(sec, len, p, hdr[p], t)) return 0;
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
