// CRC32C (Castagnoli) algebra shared by the host library and the HIP kernels.
//
// Reflected representation (zlib convention): x^0 is bit 31.  `tpi_multmodp(a, b)` is a*b
// mod P, `tpi_x8nmodp(n)` is x^(8n) mod P, so appending n zero bytes to a raw register `c`
// is `tpi_multmodp(tpi_x8nmodp(n), c)` and raw CRCs combine linearly:
//     raw(A || B) = shift(raw(A), |B|) ^ raw(B).
// The standard CRC32C (init ~0, xorout ~0) of M is raw(M) ^ shift(~0, |M|) ^ ~0.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define TPI_HD __host__ __device__
#else
#define TPI_HD
#endif

#define TPI_CRC32C_POLY 0x82F63B78u
#define TPI_ROW_LANES 256
#define TPI_ROW_BYTES (TPI_ROW_LANES * 16)  // one workgroup-wide row of 16-byte words

TPI_HD static inline uint32_t tpi_multmodp(uint32_t a, uint32_t b) {
  if (a == 0) return 0;
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ TPI_CRC32C_POLY : b >> 1;
  }
  return p;
}

TPI_HD static inline uint32_t tpi_x8nmodp(uint64_t n, const uint32_t* x2n) {
  uint32_t p = 1u << 31;  // x^0
  int k = 3;
  while (n) {
    if (n & 1) p = tpi_multmodp(x2n[k & 63], p);
    n >>= 1;
    k++;
  }
  return p;
}

// Lookup tables, built once on the host and copied to device memory; the kernels stage the
// slice/row tables into LDS.
typedef struct tpi_crc_tables {
  uint32_t slice[16][256];  // slice[j][v]: raw CRC of byte v followed by j zero bytes
  uint32_t row[4][256];     // row[j][v]: byte v at position j shifted by TPI_ROW_BYTES
  uint32_t lane_shift[TPI_ROW_LANES];  // x^(8*16*(255-l)): lane l's distance in a full row
  uint32_t x2n[64];         // x^(2^k) mod P
} tpi_crc_tables;

static inline void tpi_crc_tables_init(tpi_crc_tables* t) {
  for (uint32_t v = 0; v < 256; ++v) {
    uint32_t c = v;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ TPI_CRC32C_POLY : c >> 1;
    t->slice[0][v] = c;
  }
  for (int j = 1; j < 16; ++j)
    for (uint32_t v = 0; v < 256; ++v) {
      uint32_t c = t->slice[j - 1][v];
      t->slice[j][v] = (c >> 8) ^ t->slice[0][c & 0xff];
    }
  t->x2n[0] = 1u << 30;  // x^1
  for (int k = 1; k < 64; ++k) t->x2n[k] = tpi_multmodp(t->x2n[k - 1], t->x2n[k - 1]);
  const uint32_t xr = tpi_x8nmodp(TPI_ROW_BYTES, t->x2n);
  for (int j = 0; j < 4; ++j)
    for (uint32_t v = 0; v < 256; ++v) t->row[j][v] = tpi_multmodp(xr, v << (8 * j));
  for (int l = 0; l < TPI_ROW_LANES; ++l)
    t->lane_shift[l] = tpi_x8nmodp((uint64_t)16 * (TPI_ROW_LANES - 1 - l), t->x2n);
}

// Standard CRC32C of a whole message from its raw (zero-init, no xorout) CRC and length.
// Bank-column layout of the same tables for the CRC-only kernel (kernels.hip k_crc_tiles):
// 256 rows of 64 dwords; dword c (< 32) of row v is slice[c & 15][v], dword 32 + c is
// row[c & 3][v].  A row is 256 B, so the LDS bank of an entry is its column whatever v is.
#define TPI_CRC_COLS_WORDS (256 * 64)

static inline void tpi_crc_cols_init(const tpi_crc_tables* t, uint32_t* cols) {
  for (int v = 0; v < 256; ++v)
    for (int c = 0; c < 32; ++c) {
      cols[v * 64 + c] = t->slice[c & 15][v];
      cols[v * 64 + 32 + c] = t->row[c & 3][v];
    }
}

static inline uint32_t tpi_crc32c_finish(uint32_t raw, uint64_t len, const uint32_t* x2n) {
  return raw ^ tpi_multmodp(tpi_x8nmodp(len, x2n), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

// crc32c(A || B) from crc32c(A), crc32c(B) and |B| (standard CRCs, zlib crc32_combine).
static inline uint32_t tpi_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b,
                                          const uint32_t* x2n) {
  return tpi_multmodp(tpi_x8nmodp(len_b, x2n), crc_a) ^ crc_b;
}
