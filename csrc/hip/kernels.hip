// CDNA4 (gfx950) kernels of the checkpoint / workdir data plane.
//
//  k_stream_crc<MODE>  one 256-thread workgroup per tile of the packed stream.
//     MODE_PACK    gather tensor payloads (contiguous or strided) -> packed buffer
//     MODE_UNPACK  packed buffer -> scatter into tensors, verify tile CRC
//     MODE_CRC     CRC only (device buffer integrity digests); launched as k_crc_tiles,
//                  the bank-conflict-free column-table variant of the same math
//     MODE_COPY    tensors -> tensors (same stream layout, other pointers) + tile CRCs, with
//                  no stream buffer in between (HBM-to-HBM preemption hand-off)
//     MODE_VERIFY  gather tensors, verify tile CRCs (the hand-off's read-back check)
//   Every lane owns the 16-byte words at row*4096 + lane*16 of its tile, so each row is one
//   fully coalesced 4 KiB workgroup access (dwordx4 per lane).  The CRC32C of the tile is
//   computed without serialising lanes: lane l folds its own word stream with Horner's rule
//   (acc = acc * x^(8*4096) ^ raw16(word)), using slice-by-16 + row-shift tables staged in
//   LDS, then every lane shifts its accumulator by its distance to the tile end and the
//   workgroup XOR-reduces (wave64 shuffles + LDS across the 4 waves).
//
//  k_shard_hash  one workgroup per shard; lane l runs XXH64 over stripes l, l+256, ... so
//   every load instruction of the workgroup reads one contiguous 8 KiB span (2 x dwordx4 per
//   lane, 4 stripes in flight per lane); lanes 0..3 fold the 256 lane digests.
//
// Grid mapping: workgroup i handles tile i (linear).  The hardware deals consecutive
// workgroups round-robin over the 8 XCDs; these kernels stream every byte exactly once and
// tiles share no cache lines (tiles are 4 KiB multiples, transposes move whole 128-byte
// lines), so there is no cross-workgroup L2 reuse for an XCD-aware remap to preserve.  The
// only shared reads, the 20 KiB of CRC tables, hit in every XCD's L2 after the first wave.
//
// Reference hot paths: N2 (machine-script.sh.tpl:118-124 mtime poll),
// N4 (machine-script.sh.tpl:89,118-124 rclone data sync/restore).
#include <hip/hip_runtime.h>

#include "../common/crc32c.h"
#include "../common/xxh64.h"
#include "sysmem.h"
#include "tpi_hip.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ static inline uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

enum { MODE_PACK = 0, MODE_UNPACK = 1, MODE_CRC = 2, MODE_COPY = 3, MODE_VERIFY = 4 };
#define WG 256
#define UNROLL 8
#define LDS_WORDS (16 * 256 + 4 * 256 + WG)

__device__ static inline uint32_t raw16(const uint32_t* __restrict__ s, u32x4 w) {
  // s = slice tables [16][256]; byte k of the word goes through table 15-k.
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

__device__ static inline uint32_t shift_row(const uint32_t* __restrict__ r, uint32_t a) {
  return r[a & 0xff] ^ r[256 + ((a >> 8) & 0xff)] ^ r[512 + ((a >> 16) & 0xff)] ^
         r[768 + (a >> 24)];
}

// ---- segment (tensor) access --------------------------------------------------------------
//
// The packed stream is read/written in 16-byte words.  Per segment kind:
//   CONTIG     one dwordx4 load/store per word (nontemporal)
//   ROWS       row = rel / row_bytes; the row's base comes from the outer dims; one dwordx4
//              per word while the word stays inside an aligned row
//   TRANSPOSE  with `staged`, the bytes were already moved between tensor and stream buffer
//              by k_transpose (LDS tiles); the tile kernel only reads/keeps them there
//   otherwise  element-wise: 16/elem typed loads/stores at the view's strided offsets

struct SegCursor {
  int idx;
  uint64_t off, nbytes, ptr, next_off;
  uint32_t kind;
};

__device__ static inline void seg_load(const tpi_seg* __restrict__ segs, int n, int i,
                                       SegCursor& c) {
  c.idx = i;
  c.off = segs[i].off;
  c.nbytes = segs[i].nbytes;
  c.ptr = segs[i].ptr;
  c.kind = segs[i].kind;
  c.next_off = (i + 1 < n) ? segs[i + 1].off : ~0ull;
}

// Largest i with segs[i].off <= pos (segs sorted by off, segs[0].off == 0).
__device__ static inline int seg_find(const tpi_seg* __restrict__ segs, int n, uint64_t pos) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (segs[mid].off <= pos) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Element offset (in elements) of logical element e of a strided view.  32-bit div/mod when
// the index fits (64-bit division is a long instruction sequence on CDNA).
__device__ static inline uint64_t strided_offset(const tpi_seg& s, uint64_t e) {
  uint64_t off = 0;
  if ((e >> 32) == 0) {
    uint32_t e32 = (uint32_t)e;
    for (int d = s.ndim - 1; d >= 0; --d) {
      const uint32_t sz = (uint32_t)s.sizes[d];  // <= e's range whenever e fits 32 bits
      const uint32_t q = e32 / sz;
      off += (uint64_t)(e32 - q * sz) * (int64_t)s.strides[d];
      e32 = q;
    }
    return off;
  }
  for (int d = s.ndim - 1; d >= 0; --d) {
    uint64_t sz = (uint64_t)s.sizes[d];
    uint64_t idx = e % sz;
    e /= sz;
    off += idx * (int64_t)s.strides[d];
  }
  return off;
}

// Element-wise path: the word holds 16/E whole elements (E divides 16, words 16-aligned).
// Component arithmetic with compile-time indices only (no private arrays -> no scratch).
template <int E>
__device__ static inline uint32_t elem_bits(const uint8_t* src) {
  if (E == 1) return *src;
  if (E == 2) return *(const uint16_t*)src;
  return *(const uint32_t*)src;
}

template <int E>
__device__ static inline u32x4 gather_elems(const tpi_seg* __restrict__ segs, int idx,
                                                  uint64_t rel) {
  const tpi_seg& s = segs[idx];
  const uint8_t* base = (const uint8_t*)s.ptr;
  uint32_t u0 = 0, u1 = 0, u2 = 0, u3 = 0;
#pragma unroll
  for (int k = 0; k < 16; k += (E < 4 ? E : 4)) {
    const uint64_t q = rel + k;
    if (q >= s.nbytes) break;
    const int sub = E > 4 ? k % E : 0;  // 8/16-byte elements move as dwords
    const uint64_t off = (s.kind == TPI_SEG_CONTIG ? q - sub : strided_offset(s, q / E) * E) + sub;
    const uint32_t v = elem_bits < (E < 4 ? E : 4) > (base + off) << (8 * (k & 3));
    if (k < 4) u0 |= v; else if (k < 8) u1 |= v; else if (k < 12) u2 |= v; else u3 |= v;
  }
  return u32x4{u0, u1, u2, u3};
}

template <int E>
__device__ static inline void scatter_elems(const tpi_seg* __restrict__ segs, int idx,
                                                  uint64_t rel, u32x4 w) {
  const tpi_seg& s = segs[idx];
  uint8_t* base = (uint8_t*)s.ptr;
#pragma unroll
  for (int k = 0; k < 16; k += (E < 4 ? E : 4)) {
    const uint64_t q = rel + k;
    if (q >= s.nbytes) break;
    const int sub = E > 4 ? k % E : 0;
    const uint64_t off = (s.kind == TPI_SEG_CONTIG ? q - sub : strided_offset(s, q / E) * E) + sub;
    const uint32_t comp = k < 4 ? w.x : k < 8 ? w.y : k < 12 ? w.z : w.w;
    const uint32_t v = comp >> (8 * (k & 3));
    if (E == 1) base[off] = (uint8_t)v;
    else if (E == 2) *(uint16_t*)(base + off) = (uint16_t)v;
    else *(uint32_t*)(base + off) = v;
  }
}

// Element size as the access width; odd sizes (and unaligned bases) go byte by byte.
__device__ static inline int access_width(const tpi_seg& s) {
  const uint32_t e = s.elem;
  if (e == 0 || e > 16 || (e & (e - 1)) || (s.ptr % e)) return 1;
  return (int)e;
}

__device__ static u32x4 gather_any(const tpi_seg* __restrict__ segs, int idx, uint64_t rel) {
  switch (access_width(segs[idx])) {
    case 2: return gather_elems<2>(segs, idx, rel);
    case 4: return gather_elems<4>(segs, idx, rel);
    case 8: return gather_elems<8>(segs, idx, rel);
    case 16: return gather_elems<16>(segs, idx, rel);
    default: return gather_elems<1>(segs, idx, rel);
  }
}

__device__ static void scatter_any(const tpi_seg* __restrict__ segs, int idx, uint64_t rel,
                                   u32x4 w) {
  switch (access_width(segs[idx])) {
    case 2: scatter_elems<2>(segs, idx, rel, w); break;
    case 4: scatter_elems<4>(segs, idx, rel, w); break;
    case 8: scatter_elems<8>(segs, idx, rel, w); break;
    case 16: scatter_elems<16>(segs, idx, rel, w); break;
    default: scatter_elems<1>(segs, idx, rel, w); break;
  }
}

__device__ static inline void advance(const tpi_seg* __restrict__ segs, int n, uint64_t pos,
                                      SegCursor& c) {
  while (pos >= c.next_off) seg_load(segs, n, c.idx + 1, c);
}

// Address of a word of a ROWS segment if it can be moved as one aligned dwordx4, else 0.
__device__ static inline uint64_t rows_addr(const tpi_seg& s, uint64_t rel) {
  const uint64_t row_elems = (uint64_t)s.sizes[s.ndim - 1], row_bytes = row_elems * s.elem;
  uint64_t row;
  if (((rel | row_bytes) >> 32) == 0) row = (uint32_t)rel / (uint32_t)row_bytes;
  else row = rel / row_bytes;
  const uint64_t within = rel - row * row_bytes;
  if (within + 16 > row_bytes) return 0;
  const uint64_t outer = s.ndim == 2 ? row * (uint64_t)s.strides[0]  // matrix slice: no div
                                     : strided_offset(s, row * row_elems);
  const uint64_t addr = s.ptr + outer * s.elem + within;
  return (addr & 15) ? 0 : addr;
}

// Non-contiguous words (ROWS vectors, staged TRANSPOSE words, element-wise fallback).
__device__ static inline u32x4 gather_other(const tpi_seg* __restrict__ segs, int idx,
                                                  uint64_t rel, const uint8_t* sbuf,
                                                  bool staged) {
  const tpi_seg& s = segs[idx];
  if (s.kind == TPI_SEG_ROWS) {
    const uint64_t addr = rows_addr(s, rel);
    if (addr) return *(const u32x4*)addr;
  } else if (s.kind == TPI_SEG_TRANSPOSE && staged) {
    u32x4 w = *(const u32x4*)sbuf;
    if (rel + 16 > s.nbytes) {  // the tail word: bytes past the payload are padding (zero)
      const uint64_t keep = s.nbytes - rel;  // 1..15
      auto m = [&](int j) -> uint32_t {
        const int64_t n = (int64_t)keep - 4 * j;
        return n >= 4 ? 0xffffffffu : n <= 0 ? 0u : (1u << (8 * n)) - 1;
      };
      w.x &= m(0);
      w.y &= m(1);
      w.z &= m(2);
      w.w &= m(3);
    }
    return w;
  }
  return gather_any(segs, idx, rel);
}

__device__ static inline void scatter_other(const tpi_seg* __restrict__ segs, int idx,
                                                  uint64_t rel, u32x4 w, bool staged) {
  const tpi_seg& s = segs[idx];
  if (s.kind == TPI_SEG_ROWS) {
    const uint64_t addr = rows_addr(s, rel);
    if (addr) {
      *(u32x4*)addr = w;
      return;
    }
  } else if (s.kind == TPI_SEG_TRANSPOSE && staged) {
    return;  // k_transpose scatters this segment from the stream buffer afterwards
  }
  scatter_any(segs, idx, rel, w);
}

// `staged`: the word's bytes for TRANSPOSE segments are already at `sbuf` (stream buffer).
__device__ static inline u32x4 gather16(const tpi_seg* __restrict__ segs, const SegCursor& c,
                                        uint64_t pos, const uint8_t* sbuf, bool staged) {
  const uint64_t rel = pos - c.off;
  if (rel >= c.nbytes) return u32x4{0, 0, 0, 0};  // alignment padding
  const uint64_t addr = c.ptr + rel;
  if (c.kind == TPI_SEG_CONTIG && rel + 16 <= c.nbytes && (addr & 15) == 0)
    return __builtin_nontemporal_load((const u32x4*)addr);
  if (c.kind == TPI_SEG_TRANSPOSE && staged && rel + 16 <= c.nbytes)
    return *(const u32x4*)sbuf;  // placed by k_transpose
  return gather_other(segs, c.idx, rel, sbuf, staged);
}

__device__ static inline void scatter16(const tpi_seg* __restrict__ segs, const SegCursor& c,
                                        uint64_t pos, u32x4 w, bool staged) {
  const uint64_t rel = pos - c.off;
  if (rel >= c.nbytes) return;
  const uint64_t addr = c.ptr + rel;
  if (c.kind == TPI_SEG_CONTIG && rel + 16 <= c.nbytes && (addr & 15) == 0) {
    __builtin_nontemporal_store(w, (u32x4*)addr);  // streamed once: no L2 allocation
    return;
  }
  if (c.kind == TPI_SEG_TRANSPOSE && staged) return;  // k_transpose scatters it afterwards
  scatter_other(segs, c.idx, rel, w, staged);
}

// ---- LDS-tiled transpose for TRANSPOSE segments ------------------------------------------------
//
// A TRANSPOSE view is (B, R, C) in logical (row-major) order with memory strides (sB, 1, sC):
// memory-contiguous along R, while the stream is contiguous along C.  One 256-thread
// workgroup moves a TR(R) x TC(C) element tile (TR * TC = 4096) through LDS: the load walks
// the tile column by column with consecutive lanes on consecutive R (coalesced tensor
// reads), the store walks it row by row with consecutive lanes on consecutive C (coalesced
// stream writes).  When C <= 64 the tile spans whole logical rows (TC = C, TR = 4096 / C),
// so its stream bytes are one contiguous run -- small-C views such as channels-last conv
// weights (C = kh*kw) keep full tiles.  Each LDS column is padded to an odd number of banks,
// which keeps the transpose (nearly) free of bank conflicts (profiles/rocprof_views_round1.md).
// DIR 0: tensor -> stream buffer (before the pack kernel), DIR 1: stream buffer -> tensor
// (after the unpack kernel has verified the CRCs).  Only logical elements in [e_lo, e_hi)
// (the part of the segment inside the current chunk) are touched.

#define TP_ELEMS 4096

struct TransposeArgs {
  uint64_t ptr;      // tensor base
  uint64_t sbuf;     // address of logical element 0 of the segment in the stream buffer
  int64_t B, R, C, sB, sC;
  uint64_t e_lo, e_hi;
  uint64_t t_lo;     // first (b, r-tile) pair: b * rt + r-tile
  uint32_t ct;       // number of C tiles
  uint32_t rt;       // number of R tiles per batch
  uint32_t tr, tc;   // tile shape (tr * tc == TP_ELEMS)
};

// FULLROWS = false: 64 x 64 tiles (compile-time shape, shifts only).  FULLROWS = true: the
// tile is tr whole logical rows of C (< 64) elements, so its stream bytes are contiguous.
template <typename T, int DIR, bool FULLROWS>
__global__ __launch_bounds__(256) void k_transpose(TransposeArgs a) {
  // [tc][tr + pad]: the column stride is an odd number of 4-byte banks for every T <= 4 bytes
  constexpr uint32_t pad = sizeof(T) < 4 ? 4 / sizeof(T) : 1;
  __shared__ T tile[TP_ELEMS + 64 * 4];
  const uint32_t tr = FULLROWS ? a.tr : 64u, tc = FULLROWS ? a.tc : 64u, ld = tr + pad;
  const uint32_t n = FULLROWS ? tr * tc : (uint32_t)TP_ELEMS;
  const uint32_t trs = FULLROWS ? (uint32_t)__ffs(tr) - 1 : 6u;  // tr is a power of two
  const uint64_t pair = a.t_lo + blockIdx.x / a.ct;
  const int64_t b = (int64_t)(pair / a.rt);
  const int64_t r0 = (int64_t)(pair % a.rt) * tr;
  const int64_t c0 = (int64_t)(blockIdx.x % a.ct) * tc;
  T* tensor = (T*)a.ptr + b * a.sB;
  T* stream = (T*)a.sbuf;
  const uint64_t row0 = (uint64_t)(b * a.R) * (uint64_t)a.C;  // logical index of (b, 0, 0)
  if (DIR == 0) {
#pragma unroll 4
    for (uint32_t f = threadIdx.x; f < n; f += 256) {  // column-major: lanes along R
      const uint32_t c = f >> trs, r = f & (tr - 1);
      if (r0 + r < a.R && c0 + c < a.C) tile[c * ld + r] = tensor[r0 + r + (c0 + c) * a.sC];
    }
    __syncthreads();
#pragma unroll 4
    for (uint32_t f = threadIdx.x; f < n; f += 256) {  // row-major: lanes along C
      const uint32_t r = f / tc, c = f - r * tc;
      const uint64_t e = row0 + (uint64_t)(r0 + r) * a.C + (c0 + c);
      if (r0 + r < a.R && c0 + c < a.C && e >= a.e_lo && e < a.e_hi) stream[e] = tile[c * ld + r];
    }
  } else {
#pragma unroll 4
    for (uint32_t f = threadIdx.x; f < n; f += 256) {
      const uint32_t r = f / tc, c = f - r * tc;
      const uint64_t e = row0 + (uint64_t)(r0 + r) * a.C + (c0 + c);
      if (r0 + r < a.R && c0 + c < a.C && e >= a.e_lo && e < a.e_hi) tile[c * ld + r] = stream[e];
    }
    __syncthreads();
#pragma unroll 4
    for (uint32_t f = threadIdx.x; f < n; f += 256) {
      const uint32_t c = f >> trs, r = f & (tr - 1);
      const uint64_t e = row0 + (uint64_t)(r0 + r) * a.C + (c0 + c);
      if (r0 + r < a.R && c0 + c < a.C && e >= a.e_lo && e < a.e_hi)
        tensor[r0 + r + (c0 + c) * a.sC] = tile[c * ld + r];
    }
  }
}

template <typename T>
static void launch_transpose(const TransposeArgs& a, int dir, dim3 grid, hipStream_t stream) {
  const bool full = a.tc != 64;
  if (dir == 0) {
    if (full) hipLaunchKernelGGL((k_transpose<T, 0, true>), grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((k_transpose<T, 0, false>), grid, dim3(256), 0, stream, a);
  } else {
    if (full) hipLaunchKernelGGL((k_transpose<T, 1, true>), grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((k_transpose<T, 1, false>), grid, dim3(256), 0, stream, a);
  }
}

// ---- the tile kernel -------------------------------------------------------------------------

struct TileArgs {
  const tpi_seg* segs;
  int nseg;
  uint64_t stream_base;     // packed-stream offset of buf[0]
  uint64_t len;             // bytes of the stream covered by this launch
  uint8_t* buf;             // packed bytes of [stream_base, stream_base + len)
  uint64_t tile_bytes;      // multiple of TPI_ROW_BYTES
  const tpi_crc_tables* tables;
  uint32_t* crcs;           // indexed by global tile (stream_base / tile_bytes + blockIdx.x)
  uint32_t init_full;       // shift(~0, tile_bytes)
  uint32_t init_last;       // shift(~0, last tile length) for a short final tile
  unsigned long long* bad;  // [0] mismatching tiles, [1] first bad tile (unpack)
  const uint32_t* list;     // optional: workgroup i handles stream tile list[i] (sparse pack)
  uint64_t total;           // stream length (needed with `list`)
  int staged;               // TRANSPOSE segments are moved by k_transpose (see gather16)
  const tpi_seg* dsegs;     // MODE_COPY: destination segments (same off/nbytes as segs)
};

// Stream geometry of this workgroup's tile: (global tile, stream offset, length, buffer).
struct TileGeom {
  uint64_t gtile, gbase, len;
  uint8_t* buf;
};

__device__ static inline TileGeom tile_geom(const TileArgs& a) {
  TileGeom g;
  if (a.list) {  // sparse: compact buffer, tiles scattered over the stream
    g.gtile = a.list[blockIdx.x];
    g.gbase = g.gtile * a.tile_bytes;
    g.len = umin64(a.tile_bytes, a.total - g.gbase);
    g.buf = a.buf + (uint64_t)blockIdx.x * a.tile_bytes;
  } else {
    const uint64_t off = (uint64_t)blockIdx.x * a.tile_bytes;
    g.gtile = a.stream_base / a.tile_bytes + blockIdx.x;
    g.gbase = a.stream_base + off;
    g.len = umin64(a.tile_bytes, a.len - off);
    g.buf = a.buf + off;
  }
  return g;
}

template <int MODE>
__global__ __launch_bounds__(WG) void k_stream_crc(TileArgs a) {
  __shared__ uint32_t lds[LDS_WORDS];
  uint32_t* s_slice = lds;
  uint32_t* s_row = lds + 16 * 256;
  uint32_t* s_red = lds + 20 * 256;
  const int lane = threadIdx.x;

  {  // stage CRC tables (20 KiB) into LDS
    const u32x4* src = (const u32x4*)a.tables;
    u32x4* dst = (u32x4*)lds;
#pragma unroll
    for (int i = lane; i < 20 * 256 / 4; i += WG) dst[i] = src[i];
  }

  const TileGeom geom = tile_geom(a);
  const uint64_t tile_len = geom.len;
  const uint64_t gbase = geom.gbase;  // packed-stream offset
  uint8_t* tbuf = geom.buf;

  SegCursor cur, dcur;
  if (MODE != MODE_CRC) seg_load(a.segs, a.nseg, seg_find(a.segs, a.nseg, gbase + lane * 16), cur);
  if (MODE == MODE_COPY)
    seg_load(a.dsegs, a.nseg, seg_find(a.dsegs, a.nseg, gbase + lane * 16), dcur);
  __syncthreads();

  uint32_t acc = 0;
  uint64_t last_end = 0;
  const uint64_t nrows = (tile_len + TPI_ROW_BYTES - 1) / TPI_ROW_BYTES;
  uint64_t row = 0;
  // Full groups of UNROLL rows where every lane has a word (no bounds checks).
  const uint64_t full_rows = tile_len / TPI_ROW_BYTES;
  for (; row + UNROLL <= full_rows; row += UNROLL) {
    u32x4 w[UNROLL];
    uint32_t kept = 0;  // bit u: word u is a staged TRANSPOSE word already in place
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t rel = (row + u) * TPI_ROW_BYTES + lane * 16;
      if (MODE == MODE_PACK) {
        advance(a.segs, a.nseg, gbase + rel, cur);
        w[u] = gather16(a.segs, cur, gbase + rel, tbuf + rel, a.staged);
        kept |= (cur.kind == TPI_SEG_TRANSPOSE && gbase + rel + 16 <= cur.off + cur.nbytes ? 1u
                                                                                      : 0u)
                << u;
      } else if (MODE == MODE_COPY || MODE == MODE_VERIFY) {
        advance(a.segs, a.nseg, gbase + rel, cur);
        w[u] = gather16(a.segs, cur, gbase + rel, nullptr, false);
      } else {
        w[u] = __builtin_nontemporal_load((const u32x4*)(tbuf + rel));
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const uint64_t rel = (row + u) * TPI_ROW_BYTES + lane * 16;
      if (MODE == MODE_PACK) {
        // staged TRANSPOSE words are already in place (except a tail word's padding)
        if (!(a.staged && ((kept >> u) & 1u)))
          __builtin_nontemporal_store(w[u], (u32x4*)(tbuf + rel));
      } else if (MODE == MODE_UNPACK) {
        advance(a.segs, a.nseg, gbase + rel, cur);
        scatter16(a.segs, cur, gbase + rel, w[u], a.staged);
      } else if (MODE == MODE_COPY) {
        advance(a.dsegs, a.nseg, gbase + rel, dcur);
        scatter16(a.dsegs, dcur, gbase + rel, w[u], false);
      }
      acc = shift_row(s_row, acc) ^ raw16(s_slice, w[u]);
    }
    last_end = (row + UNROLL - 1) * TPI_ROW_BYTES + lane * 16 + 16;
  }
  for (; row < nrows; ++row) {  // remainder rows, possibly partial
    const uint64_t rel = row * TPI_ROW_BYTES + lane * 16;
    if (rel < tile_len) {
      u32x4 w;
      if (MODE == MODE_PACK) {
        advance(a.segs, a.nseg, gbase + rel, cur);
        w = gather16(a.segs, cur, gbase + rel, tbuf + rel, a.staged);
        __builtin_nontemporal_store(w, (u32x4*)(tbuf + rel));
      } else if (MODE == MODE_COPY || MODE == MODE_VERIFY) {
        advance(a.segs, a.nseg, gbase + rel, cur);
        w = gather16(a.segs, cur, gbase + rel, nullptr, false);
        if (MODE == MODE_COPY) {
          advance(a.dsegs, a.nseg, gbase + rel, dcur);
          scatter16(a.dsegs, dcur, gbase + rel, w, false);
        }
      } else {
        w = __builtin_nontemporal_load((const u32x4*)(tbuf + rel));
        if (MODE == MODE_UNPACK) {
          advance(a.segs, a.nseg, gbase + rel, cur);
          scatter16(a.segs, cur, gbase + rel, w, a.staged);
        }
      }
      acc = shift_row(s_row, acc) ^ raw16(s_slice, w);
      last_end = rel + 16;
    }
  }

  // Shift each lane's accumulator to the end of the tile and XOR-reduce.
  uint32_t contrib = 0;
  if (last_end) {
    const uint64_t dist = tile_len - last_end;
    uint32_t k = (tile_len % TPI_ROW_BYTES == 0) ? a.tables->lane_shift[lane]
                                                 : tpi_x8nmodp(dist, a.tables->x2n);
    contrib = tpi_multmodp(k, acc);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) contrib ^= __shfl_xor(contrib, o, 64);
  if ((lane & 63) == 0) s_red[lane >> 6] = contrib;
  __syncthreads();
  if (lane == 0) {
    uint32_t raw = s_red[0] ^ s_red[1] ^ s_red[2] ^ s_red[3];
    const uint32_t init = (tile_len == a.tile_bytes) ? a.init_full : a.init_last;
    const uint32_t crc = raw ^ init ^ 0xFFFFFFFFu;
    const uint64_t gtile = geom.gtile;
    if (MODE == MODE_UNPACK || MODE == MODE_VERIFY) {
      if (crc != tpi_sys_load(&a.crcs[gtile])) {
        atomicAdd(&a.bad[0], 1ull);
        atomicMin(&a.bad[1], (unsigned long long)gtile);
      }
    } else {
      tpi_sys_store(&a.crcs[gtile], crc);
    }
  }
}

// ---- CRC-only tiles: bank-conflict-free column tables ---------------------------------------
//
// MODE_CRC of k_stream_crc was bound by LDS bank conflicts (profiles/crc_lds_round2.md): a
// lookup's index is a data byte, so the 32 lanes of a ds_read_b32 group hit random banks and
// a group costs ~3.5 cycles.  k_crc_tiles reads the column layout of the same tables
// (crc32c.h tpi_crc_cols_init: 256 rows x 256 B, every table copy in ONE bank column):
//   * at unrolled step j of a word, lane l uses column (j + l) mod 32 -- a permutation of the
//     32 banks over each lane group -- i.e. slice table (j + l) mod 16;
//   * each lane first rotates its 16-byte word left by (l mod 16) bytes (8 v_cndmask + 4
//     v_alignbyte on lane-constant masks), so step j always needs byte 15 - j;
//   * the LDS byte address (data byte) << 8 | (column << 2) is one v_perm_b32 of the data
//     dword and a register packing four of the lane's columns; the row shift picks the
//     accumulator byte with a lane-constant perm selector and the row columns (+128 B).
// Every lookup is conflict-free at 1 VALU + 1 xor, as many as the production layout.  512
// threads per workgroup (two tiles, one per half) share the 64 KiB of tables: 16 waves per
// CU at ~110 VGPRs.  Grid-stride over tile pairs, tables staged once per workgroup.
// 8 GB of 1 MiB tiles on MI355X: 4.30 -> 6.63 TB/s (scripts/exp/crc_cf.hip, same math).

#define CRC_WG 512

struct ColLane {
  bool m1, m2;          // rotate the word by one / two dwords
  uint32_t s;           // then by s bytes (v_alignbyte)
  uint32_t colpack[4];  // byte i of colpack[k]: ((4k + i + l) mod 32) * 4
  uint32_t selR[4];     // row step j: byte0 <- colpack[0] byte j, byte1 <- acc byte (j + l) & 3
};

__device__ static inline ColLane col_lane(int lane) {
  ColLane m;
  const int l32 = lane & 31, r = lane & 15;
  const int q2 = ((r + 3) >> 2) & 3;
  m.m1 = q2 & 1;
  m.m2 = q2 & 2;
  m.s = (uint32_t)((4 - (r & 3)) & 3);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) c |= (uint32_t)(((4 * k + i + l32) & 31) * 4) << (8 * i);
    m.colpack[k] = c;
    m.selR[k] = 0x0C0C0000u | ((4u + (uint32_t)((k + l32) & 3)) << 8) | (uint32_t)k;
  }
  return m;
}

__device__ static inline uint32_t col_at(const uint32_t* t, uint32_t byte_off) {
  return *(const uint32_t*)((const char*)t + byte_off);
}

__device__ static inline uint32_t raw16_col(const uint32_t* t, const ColLane& m, u32x4 w) {
  const uint32_t t0 = m.m1 ? w.w : w.x, t1 = m.m1 ? w.x : w.y, t2 = m.m1 ? w.y : w.z,
                 t3 = m.m1 ? w.z : w.w;
  const uint32_t x0 = m.m2 ? t2 : t0, x1 = m.m2 ? t3 : t1, x2 = m.m2 ? t0 : t2,
                 x3 = m.m2 ? t1 : t3;
  uint32_t R[4];
  R[0] = __builtin_amdgcn_alignbyte(x1, x0, m.s);
  R[1] = __builtin_amdgcn_alignbyte(x2, x1, m.s);
  R[2] = __builtin_amdgcn_alignbyte(x3, x2, m.s);
  R[3] = __builtin_amdgcn_alignbyte(x0, x3, m.s);
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int pos = 15 - j;
    const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(pos & 3)) << 8) | (uint32_t)(j & 3);
    c ^= col_at(t, __builtin_amdgcn_perm(R[pos >> 2], m.colpack[j >> 2], sel));
  }
  return c;
}

__device__ static inline uint32_t shift_row_col(const uint32_t* t, const ColLane& m, uint32_t a) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) c ^= col_at(t + 32, __builtin_amdgcn_perm(a, m.colpack[0], m.selR[j]));
  return c;
}

__global__ __launch_bounds__(CRC_WG) void k_crc_tiles(TileArgs a) {
  __shared__ uint32_t lds[TPI_CRC_COLS_WORDS + 2 * (WG / 64)];  // static: no base add per lookup
  uint32_t* s_red = lds + TPI_CRC_COLS_WORDS;
  const int tid = threadIdx.x, lane = tid & (WG - 1);
  // wave-uniform, and made scalar: tile geometry and row loops then run on SGPRs instead
  // of a divergent VGPR loop (5.5 -> 6.x TB/s)
  const int half = __builtin_amdgcn_readfirstlane(tid) / WG;
  {
    const u32x4* src = (const u32x4*)(a.tables + 1);  // column layout follows the struct
    u32x4* dst = (u32x4*)lds;
    for (int i = tid; i < TPI_CRC_COLS_WORDS / 4; i += CRC_WG) dst[i] = src[i];
  }
  const ColLane m = col_lane(lane);
  __syncthreads();
  const uint64_t ntiles = (a.len + a.tile_bytes - 1) / a.tile_bytes;
  for (uint64_t pair = blockIdx.x; pair * 2 < ntiles; pair += gridDim.x) {
    const uint64_t t = pair * 2 + half;
    uint32_t contrib = 0;
    uint64_t tile_len = 0;
    if (t < ntiles) {
      const uint64_t off = t * a.tile_bytes;
      tile_len = umin64(a.tile_bytes, a.len - off);
      const uint8_t* tbuf = a.buf + off;
      uint32_t acc = 0;
      uint64_t last_end = 0, row = 0;
      const uint64_t nrows = (tile_len + TPI_ROW_BYTES - 1) / TPI_ROW_BYTES;
      const uint64_t full_rows = tile_len / TPI_ROW_BYTES;
      for (; row + UNROLL <= full_rows; row += UNROLL) {
        u32x4 w[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
          w[u] = __builtin_nontemporal_load(
              (const u32x4*)(tbuf + (row + u) * TPI_ROW_BYTES + lane * 16));
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc = shift_row_col(lds, m, acc) ^ raw16_col(lds, m, w[u]);
        last_end = (row + UNROLL - 1) * TPI_ROW_BYTES + lane * 16 + 16;
      }
      for (; row < nrows; ++row) {  // remainder rows, possibly partial
        const uint64_t rel = row * TPI_ROW_BYTES + lane * 16;
        if (rel < tile_len) {
          const u32x4 w = __builtin_nontemporal_load((const u32x4*)(tbuf + rel));
          acc = shift_row_col(lds, m, acc) ^ raw16_col(lds, m, w);
          last_end = rel + 16;
        }
      }
      if (last_end) {
        const uint32_t k = (tile_len % TPI_ROW_BYTES == 0)
                               ? a.tables->lane_shift[lane]
                               : tpi_x8nmodp(tile_len - last_end, a.tables->x2n);
        contrib = tpi_multmodp(k, acc);
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) contrib ^= __shfl_xor(contrib, o, 64);
    __syncthreads();  // s_red reuse across pairs
    if ((tid & 63) == 0) s_red[tid >> 6] = contrib;
    __syncthreads();
    if (lane == 0 && t < ntiles) {
      const uint32_t* r = s_red + (WG / 64) * half;
      const uint32_t init = (tile_len == a.tile_bytes) ? a.init_full : a.init_last;
      tpi_sys_store(&a.crcs[a.stream_base / a.tile_bytes + t],
                    r[0] ^ r[1] ^ r[2] ^ r[3] ^ init ^ 0xFFFFFFFFu);
    }
  }
}

// ---- striped XXH64 shard hash ----------------------------------------------------------------

__global__ __launch_bounds__(WG) void k_shard_hash(const uint8_t* __restrict__ data,
                                                   uint64_t nbytes, uint64_t shard_bytes,
                                                   uint64_t seed, uint64_t* __restrict__ out) {
  __shared__ uint64_t dig[TPI_HASH_LANES];
  const int lane = threadIdx.x;
  const uint64_t base = (uint64_t)blockIdx.x * shard_bytes;
  const uint64_t len = umin64(shard_bytes, nbytes - base);
  const uint8_t* d = data + base;
  const uint64_t full = len / TPI_HASH_STRIPE;
  const uint32_t rem = (uint32_t)(len % TPI_HASH_STRIPE);
  const uint64_t nfull = full > (uint64_t)lane ? (full - lane + WG - 1) / WG : 0;
  const bool owns_tail = rem && (full % WG) == (uint64_t)lane;
  const uint64_t mylen = nfull * TPI_HASH_STRIPE + (owns_tail ? rem : 0);

  uint64_t h;
  if (mylen >= 32) {
    uint64_t v1 = seed + TPI_XXH_P1 + TPI_XXH_P2, v2 = seed + TPI_XXH_P2, v3 = seed,
             v4 = seed - TPI_XXH_P1;
    const u32x4* p = (const u32x4*)(d + (uint64_t)lane * TPI_HASH_STRIPE);
    const uint64_t step = WG * TPI_HASH_STRIPE / 16;  // in u32x4 units
    uint64_t j = 0;
    for (; j + 4 <= nfull; j += 4) {
      u32x4 w[8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        w[2 * u] = __builtin_nontemporal_load(p + (j + u) * step);
        w[2 * u + 1] = __builtin_nontemporal_load(p + (j + u) * step + 1);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v1 = tpi_xxh_round(v1, ((uint64_t)w[2 * u].y << 32) | w[2 * u].x);
        v2 = tpi_xxh_round(v2, ((uint64_t)w[2 * u].w << 32) | w[2 * u].z);
        v3 = tpi_xxh_round(v3, ((uint64_t)w[2 * u + 1].y << 32) | w[2 * u + 1].x);
        v4 = tpi_xxh_round(v4, ((uint64_t)w[2 * u + 1].w << 32) | w[2 * u + 1].z);
      }
    }
    for (; j < nfull; ++j) {
      u32x4 a = p[j * step], b = p[j * step + 1];
      v1 = tpi_xxh_round(v1, ((uint64_t)a.y << 32) | a.x);
      v2 = tpi_xxh_round(v2, ((uint64_t)a.w << 32) | a.z);
      v3 = tpi_xxh_round(v3, ((uint64_t)b.y << 32) | b.x);
      v4 = tpi_xxh_round(v4, ((uint64_t)b.w << 32) | b.z);
    }
    h = tpi_xxh_converge(v1, v2, v3, v4);
  } else {
    h = seed + TPI_XXH_P5;
  }
  h += mylen;
  // The tail (< 32 bytes, one lane per shard) is read straight from global memory.
  dig[lane] = tpi_xxh_finish(h, d + full * TPI_HASH_STRIPE, owns_tail ? rem : 0);
  __syncthreads();

  // XXH64 over the 2048-byte digest array: 64 stripes of 4 words; lane k<4 owns word k.
  if (lane < 64) {
    uint64_t v = 0;
    if (lane < 4) {
      v = lane == 0 ? seed + TPI_XXH_P1 + TPI_XXH_P2
        : lane == 1 ? seed + TPI_XXH_P2
        : lane == 2 ? seed
                    : seed - TPI_XXH_P1;
      for (int s = 0; s < TPI_HASH_LANES / 4; ++s) v = tpi_xxh_round(v, dig[4 * s + lane]);
    }
    const uint64_t v1 = __shfl(v, 0, 64), v2 = __shfl(v, 1, 64), v3 = __shfl(v, 2, 64),
                   v4 = __shfl(v, 3, 64);
    if (lane == 0) {
      uint64_t hh = tpi_xxh_converge(v1, v2, v3, v4) + (uint64_t)(TPI_HASH_LANES * 8);
      out[blockIdx.x] = tpi_xxh_avalanche(hh);
    }
  }
}

// ---- incremental checkpoints: per-tile digests gathered from the tensors -----------------------
//
// 64-bit change-detection digest of every tile of the *virtual* packed stream, read straight
// from the tensors (nothing is written).  Lane l folds its words (row*4096 + 16l, the same
// coalesced layout as the tile kernel) with XXH64 rounds from a lane-distinct seed; the tile
// digest is the XOR of the avalanched lane states, mixed with the tile length.  It is a
// private format (only compared with itself), so it needs no host reference beyond tests.

//
// The same digest drives the HBM hand-off's fused copy (HASH_COPY: every word gathered from the
// predecessor's tensors is also scattered into the successor's, and the tile digest of what
// was read is recorded) and its read-back check (HASH_VERIFY: the successor's tensors are
// hashed again and compared).  No table lookups: where the CRC32C verify is bound by its LDS
// lookups at ~4.3 TB/s, this reads at the ~6 TB/s class of k_shard_hash
// (profiles/handoff_hash_round3.md).  Workgroup i handles tile tile0 + i.
//
// HASH_COPY_CHECK copies like HASH_COPY and checks the destination inline: each lane reads back
// the words it stored one row group earlier (the lag keeps the read-back off the stores'
// latency) and compares them with the words it copied, so the destination is verified without
// a second pass over HBM -- the read-back mostly hits the caches the stores just went through.
// Overlapping destinations, the one fault an immediate read-back cannot see (a later writer
// could still overwrite a checked word), are refused on the host before the launch
// (tpi_copy_segments).
enum { HASH_ONLY = 0, HASH_COPY = 1, HASH_VERIFY = 2, HASH_COPY_CHECK = 3 };

template <int KIND, int U = UNROLL>
__global__ __launch_bounds__(WG) void k_stream_hash(const tpi_seg* __restrict__ segs,
                                                    const tpi_seg* __restrict__ dsegs, int nseg,
                                                    uint64_t tile0, uint64_t total,
                                                    uint64_t tile_bytes, uint64_t seed,
                                                    uint64_t* __restrict__ out,
                                                    unsigned long long* __restrict__ bad) {
  constexpr bool COPY = KIND == HASH_COPY || KIND == HASH_COPY_CHECK;
  constexpr bool CHECK = KIND == HASH_COPY_CHECK;
  __shared__ uint64_t red[WG / 64];
  __shared__ int mism[WG / 64];
  const int lane = threadIdx.x;
  const uint64_t gtile = tile0 + blockIdx.x;
  const uint64_t gbase = gtile * tile_bytes;
  const uint64_t len = umin64(tile_bytes, total - gbase);
  SegCursor cur, dcur, rcur;
  seg_load(segs, nseg, seg_find(segs, nseg, gbase + lane * 16), cur);
  if (COPY) seg_load(dsegs, nseg, seg_find(dsegs, nseg, gbase + lane * 16), dcur);
  if (CHECK) rcur = dcur;
  // two independent round chains per lane (low and high 8 bytes of each word): a single
  // chain of dependent 64-bit multiplies left the kernel latency-bound (4.8 TB/s)
  uint64_t va = seed + (uint64_t)(lane + 1) * TPI_XXH_P1, vb = va ^ TPI_XXH_P2;
  uint64_t nwords = 0;
  uint32_t diff = 0;  // CHECK: OR of (read back ^ copied) over this lane's words
  const uint64_t full_rows = len / TPI_ROW_BYTES;
  uint64_t row = 0;
  u32x4 prev[CHECK ? U : 1];
  bool have_prev = false;
  for (; row + U <= full_rows; row += U) {
    u32x4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t pos = gbase + (row + u) * TPI_ROW_BYTES + lane * 16;
      advance(segs, nseg, pos, cur);
      w[u] = gather16(segs, cur, pos, nullptr, false);
    }
    if (CHECK && have_prev) {
      __asm__ volatile("" ::: "memory");  // the stores below were issued: really read them back
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t pos = gbase + (row - U + u) * TPI_ROW_BYTES + lane * 16;
        advance(dsegs, nseg, pos, rcur);
        const u32x4 r = gather16(dsegs, rcur, pos, nullptr, false);
        diff |= (r.x ^ prev[u].x) | (r.y ^ prev[u].y) | (r.z ^ prev[u].z) | (r.w ^ prev[u].w);
      }
    }
    if (COPY) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t pos = gbase + (row + u) * TPI_ROW_BYTES + lane * 16;
        advance(dsegs, nseg, pos, dcur);
        scatter16(dsegs, dcur, pos, w[u], false);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va = tpi_xxh_round(va, ((uint64_t)w[u].y << 32) | w[u].x);
      vb = tpi_xxh_round(vb, ((uint64_t)w[u].w << 32) | w[u].z);
      if (CHECK) prev[u] = w[u];
    }
    if (CHECK) have_prev = true;
    nwords += U;
  }
  if (CHECK && have_prev) {  // the last full group
    __asm__ volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t pos = gbase + (row - U + u) * TPI_ROW_BYTES + lane * 16;
      advance(dsegs, nseg, pos, rcur);
      const u32x4 r = gather16(dsegs, rcur, pos, nullptr, false);
      diff |= (r.x ^ prev[u].x) | (r.y ^ prev[u].y) | (r.z ^ prev[u].z) | (r.w ^ prev[u].w);
    }
  }
  for (uint64_t rel = row * TPI_ROW_BYTES + lane * 16; rel < len; rel += TPI_ROW_BYTES) {
    advance(segs, nseg, gbase + rel, cur);
    const u32x4 w = gather16(segs, cur, gbase + rel, nullptr, false);
    if (COPY) {
      advance(dsegs, nseg, gbase + rel, dcur);
      scatter16(dsegs, dcur, gbase + rel, w, false);
    }
    if (CHECK) {
      __asm__ volatile("" ::: "memory");
      advance(dsegs, nseg, gbase + rel, rcur);
      const u32x4 r = gather16(dsegs, rcur, gbase + rel, nullptr, false);
      diff |= (r.x ^ w.x) | (r.y ^ w.y) | (r.z ^ w.z) | (r.w ^ w.w);
    }
    va = tpi_xxh_round(va, ((uint64_t)w.y << 32) | w.x);
    vb = tpi_xxh_round(vb, ((uint64_t)w.w << 32) | w.z);
    ++nwords;
  }
  uint64_t h = tpi_xxh_avalanche(va + ((vb << 31) | (vb >> 33)) + nwords * 16);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) h ^= __shfl_xor(h, o, 64);
  if ((lane & 63) == 0) red[lane >> 6] = h;
  if (CHECK) {
    const int any = __any(diff != 0);  // wave vote
    if ((lane & 63) == 0) mism[lane >> 6] = any;
  }
  __syncthreads();
  if (lane == 0) {
    const uint64_t digest = tpi_xxh_avalanche(red[0] ^ red[1] ^ red[2] ^ red[3] ^ len);
    if (KIND == HASH_VERIFY) {
      if (digest != out[gtile]) {
        atomicAdd(&bad[0], 1ull);
        atomicMin(&bad[1], (unsigned long long)gtile);
      }
    } else {
      out[gtile] = digest;
      if (CHECK && (mism[0] | mism[1] | mism[2] | mism[3])) {
        atomicAdd(&bad[0], 1ull);
        atomicMin(&bad[1], (unsigned long long)gtile);
      }
    }
  }
}

// Compare digests with the previous sync, append dirty tile indices, remember the new ones.
__global__ __launch_bounds__(256) void k_dirty_tiles(const uint64_t* __restrict__ hash,
                                                     uint64_t* __restrict__ prev, uint64_t n,
                                                     int all, uint32_t* __restrict__ idx,
                                                     unsigned int* __restrict__ count) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = hash[i];
  if (all || h != prev[i]) {
    idx[atomicAdd(count, 1u)] = (uint32_t)i;
    prev[i] = h;
  }
}

// ---- launch helpers (used by engine.hip) -----------------------------------------------------

extern "C" hipError_t tpi_launch_stream_crc(int mode, const tpi_seg* segs, int nseg,
                                            uint64_t stream_base, uint64_t len, void* buf,
                                            uint64_t tile_bytes, const tpi_crc_tables* tables,
                                            uint32_t* crcs, uint32_t init_full,
                                            uint32_t init_last, unsigned long long* bad,
                                            int staged, hipStream_t stream) {
  if (len == 0) return hipSuccess;
  TileArgs a;
  a.segs = segs;
  a.nseg = nseg;
  a.stream_base = stream_base;
  a.len = len;
  a.buf = (uint8_t*)buf;
  a.tile_bytes = tile_bytes;
  a.tables = tables;
  a.crcs = crcs;
  a.init_full = init_full;
  a.init_last = init_last;
  a.bad = bad;
  a.list = nullptr;
  a.total = 0;
  a.staged = staged;
  a.dsegs = nullptr;
  const uint64_t ntiles = (len + tile_bytes - 1) / tile_bytes;
  dim3 grid((unsigned)ntiles), block(WG);
  switch (mode) {
    case MODE_PACK: hipLaunchKernelGGL(k_stream_crc<MODE_PACK>, grid, block, 0, stream, a); break;
    case MODE_UNPACK:
      hipLaunchKernelGGL(k_stream_crc<MODE_UNPACK>, grid, block, 0, stream, a);
      break;
    default: {
      // CRC only: column-table kernel, two tiles per workgroup, grid-stride over the pairs
      // with two workgroups per CU resident (64 KiB LDS each).
      static int cu_count[64];  // per device, queried once (the attribute query is not free)
      int dev = 0, cus = 256;
      if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
        if (!__atomic_load_n(&cu_count[dev], __ATOMIC_RELAXED)) {
          int c = 0;
          if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
              c > 0)
            __atomic_store_n(&cu_count[dev], c, __ATOMIC_RELAXED);
        }
        if (cu_count[dev]) cus = cu_count[dev];
      }
      const uint64_t pairs = (ntiles + 1) / 2;
      const unsigned g = (unsigned)(pairs < (uint64_t)cus * 2 ? pairs : (uint64_t)cus * 2);
      hipLaunchKernelGGL(k_crc_tiles, dim3(g), dim3(CRC_WG), 0, stream, a);
      break;
    }
  }
  return hipGetLastError();
}

// MODE_COPY (dst != nullptr: src tensors -> dst tensors + tile CRCs into `crcs`) or
// MODE_VERIFY (dst == nullptr: gather `src`, count tiles whose CRC differs from `crcs`) over
// stream bytes [stream_base, stream_base + len).  No stream buffer; TRANSPOSE segments take
// the element-wise path.
extern "C" hipError_t tpi_launch_stream_copy(const tpi_seg* src, const tpi_seg* dst, int nseg,
                                             uint64_t stream_base, uint64_t len,
                                             uint64_t tile_bytes, const tpi_crc_tables* tables,
                                             uint32_t* crcs, uint32_t init_full,
                                             uint32_t init_last, unsigned long long* bad,
                                             hipStream_t stream) {
  if (len == 0) return hipSuccess;
  TileArgs a;
  a.segs = src;
  a.nseg = nseg;
  a.stream_base = stream_base;
  a.len = len;
  a.buf = nullptr;
  a.tile_bytes = tile_bytes;
  a.tables = tables;
  a.crcs = crcs;
  a.init_full = init_full;
  a.init_last = init_last;
  a.bad = bad;
  a.list = nullptr;
  a.total = 0;
  a.staged = 0;
  a.dsegs = dst;
  const dim3 grid((unsigned)((len + tile_bytes - 1) / tile_bytes)), block(WG);
  if (dst) hipLaunchKernelGGL(k_stream_crc<MODE_COPY>, grid, block, 0, stream, a);
  else hipLaunchKernelGGL(k_stream_crc<MODE_VERIFY>, grid, block, 0, stream, a);
  return hipGetLastError();
}

extern "C" hipError_t tpi_launch_shard_hash(const void* data, uint64_t nbytes,
                                            uint64_t shard_bytes, uint64_t seed, uint64_t* out,
                                            hipStream_t stream) {
  if (nbytes == 0) return hipSuccess;
  const uint64_t nshards = (nbytes + shard_bytes - 1) / shard_bytes;
  hipLaunchKernelGGL(k_shard_hash, dim3((unsigned)nshards), dim3(WG), 0, stream,
                     (const uint8_t*)data, nbytes, shard_bytes, seed, out);
  return hipGetLastError();
}

// Pack only the stream tiles listed in `list` (device, n entries) into `buf` compactly
// (entry i -> buf + i * tile_bytes), writing their CRCs at crcs[list[i]].
extern "C" hipError_t tpi_launch_pack_list(const tpi_seg* segs, int nseg, uint64_t total,
                                           const uint32_t* list, uint32_t n, void* buf,
                                           uint64_t tile_bytes, const tpi_crc_tables* tables,
                                           uint32_t* crcs, uint32_t init_full,
                                           uint32_t init_last, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  TileArgs a;
  a.segs = segs;
  a.nseg = nseg;
  a.stream_base = 0;
  a.len = total;
  a.buf = (uint8_t*)buf;
  a.tile_bytes = tile_bytes;
  a.tables = tables;
  a.crcs = crcs;
  a.init_full = init_full;
  a.init_last = init_last;
  a.bad = nullptr;
  a.list = list;
  a.dsegs = nullptr;
  a.total = total;
  a.staged = 0;
  hipLaunchKernelGGL(k_stream_crc<MODE_PACK>, dim3(n), dim3(WG), 0, stream, a);
  return hipGetLastError();
}

extern "C" hipError_t tpi_launch_stream_hash(const tpi_seg* segs, int nseg, uint64_t total,
                                             uint64_t tile_bytes, uint64_t seed, uint64_t* out,
                                             hipStream_t stream) {
  if (total == 0) return hipSuccess;
  const uint64_t ntiles = (total + tile_bytes - 1) / tile_bytes;
  hipLaunchKernelGGL(k_stream_hash<HASH_ONLY>, dim3((unsigned)ntiles), dim3(WG), 0, stream,
                     segs, nullptr, nseg, (uint64_t)0, total, tile_bytes, seed, out, nullptr);
  return hipGetLastError();
}

// Hand-off over the stream bytes [stream_base, stream_base + len) (tile aligned) of a plan
// whose stream is `total` bytes: dst != nullptr copies src -> dst and records the tile
// digests of what was read into `digests` (indexed by global tile) -- with `bad` also reading
// every stored word back (HASH_COPY_CHECK); dst == nullptr re-hashes src and counts tiles
// whose digest differs (bad[0]; bad[1] = first such tile).
extern "C" hipError_t tpi_launch_stream_copy_hash(const tpi_seg* src, const tpi_seg* dst,
                                                  int nseg, uint64_t stream_base, uint64_t len,
                                                  uint64_t total, uint64_t tile_bytes,
                                                  uint64_t seed, uint64_t* digests,
                                                  unsigned long long* bad, hipStream_t stream) {
  if (len == 0) return hipSuccess;
  if (stream_base % tile_bytes || stream_base + len > total) return hipErrorInvalidValue;
  const uint64_t tile0 = stream_base / tile_bytes;
  const dim3 grid((unsigned)((len + tile_bytes - 1) / tile_bytes)), block(WG);
  // rows in flight per lane (16 B each; TPI_HANDOFF_UNROLL 2, 4, 8 or 16).  2 is the fastest
  // on MI355X: more waves resident beat more bytes per wave -- 100 GB copy + read-back 49.7 ms
  // at 2, 51.7 at 4; 32 GB copy 11.7 ms at 4, 12.5 at 8, 22.2 at 16
  // (profiles/round5/handoff_kernels.md)
  static const int unroll = [] {
    const char* v = getenv("TPI_HANDOFF_UNROLL");
    return v && atoi(v) == 16 ? 16 : v && atoi(v) == 8 ? 8 : v && atoi(v) == 4 ? 4 : 2;
  }();
#define TPI_HASH_LAUNCH(UU)                                                                   \
  if (dst && bad)                                                                            \
    hipLaunchKernelGGL((k_stream_hash<HASH_COPY_CHECK, UU>), grid, block, 0, stream, src, dst, \
                       nseg, tile0, total, tile_bytes, seed, digests, bad);                   \
  else if (dst)                                                                              \
    hipLaunchKernelGGL((k_stream_hash<HASH_COPY, UU>), grid, block, 0, stream, src, dst, nseg, \
                       tile0, total, tile_bytes, seed, digests, bad);                         \
  else                                                                                       \
    hipLaunchKernelGGL((k_stream_hash<HASH_VERIFY, UU>), grid, block, 0, stream, src, nullptr, \
                       nseg, tile0, total, tile_bytes, seed, digests, bad);
  if (unroll == 16) {
    TPI_HASH_LAUNCH(16)
  } else if (unroll == 8) {
    TPI_HASH_LAUNCH(8)
  } else if (unroll == 2) {
    TPI_HASH_LAUNCH(2)
  } else {
    TPI_HASH_LAUNCH(4)
  }
#undef TPI_HASH_LAUNCH
  return hipGetLastError();
}

extern "C" hipError_t tpi_launch_dirty_tiles(const uint64_t* hash, uint64_t* prev, uint64_t n,
                                             int all, uint32_t* idx, unsigned int* count,
                                             hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_dirty_tiles, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     hash, prev, n, all, idx, count);
  return hipGetLastError();
}

// Transposes of the TRANSPOSE segments (host descriptors) overlapping the stream window
// [base, base + len) whose bytes live at `buf` (buf[0] = stream byte `base`).
extern "C" hipError_t tpi_launch_transposes(const tpi_seg* host_segs, int nseg, uint64_t base,
                                            uint64_t len, void* buf, int dir,
                                            hipStream_t stream) {
  if (!host_segs) return hipSuccess;
  for (int i = 0; i < nseg; ++i) {
    const tpi_seg& s = host_segs[i];
    if (s.kind != TPI_SEG_TRANSPOSE) continue;
    const uint64_t lo = s.off > base ? s.off : base;
    const uint64_t hi = s.off + s.nbytes < base + len ? s.off + s.nbytes : base + len;
    if (lo >= hi) continue;
    TransposeArgs a;
    a.ptr = s.ptr;
    a.sbuf = (uint64_t)buf + s.off - base;  // may point before buf: only [e_lo, e_hi) is used
    if (s.ndim == 3) {
      a.B = s.sizes[0]; a.sB = s.strides[0]; a.R = s.sizes[1]; a.C = s.sizes[2];
      a.sC = s.strides[2];
    } else {
      a.B = 1; a.sB = 0; a.R = s.sizes[0]; a.C = s.sizes[1]; a.sC = s.strides[1];
    }
    a.e_lo = (lo - s.off) / s.elem;
    a.e_hi = (hi - s.off + s.elem - 1) / s.elem;
    // tile shape: whole rows when C < 64 (TC = C, TR = largest power of two with
    // TR * C <= 4096), else 64 x 64
    a.tc = a.C < 64 ? (uint32_t)a.C : 64u;
    a.tr = 64;
    while (a.tc < 64 && a.tr * 2 * a.tc <= TP_ELEMS) a.tr *= 2;
    a.ct = (uint32_t)((a.C + a.tc - 1) / a.tc);
    a.rt = (uint32_t)((a.R + a.tr - 1) / a.tr);
    const uint64_t lr_lo = a.e_lo / a.C, lr_hi = (a.e_hi - 1) / a.C;  // logical rows b*R + r
    const uint64_t b_lo = lr_lo / a.R, b_hi = lr_hi / a.R;
    a.t_lo = b_lo * a.rt + (lr_lo - b_lo * a.R) / a.tr;
    const uint64_t t_hi = b_hi * a.rt + (lr_hi - b_hi * a.R) / a.tr;
    const uint64_t blocks = (t_hi - a.t_lo + 1) * a.ct;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    const dim3 grid((unsigned)blocks);
    switch (s.elem) {
      case 1: launch_transpose<uint8_t>(a, dir, grid, stream); break;
      case 2: launch_transpose<uint16_t>(a, dir, grid, stream); break;
      case 4: launch_transpose<uint32_t>(a, dir, grid, stream); break;
      case 8: launch_transpose<uint64_t>(a, dir, grid, stream); break;
      default: return hipErrorInvalidValue;  // the host only emits TRANSPOSE for 1/2/4/8
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}
