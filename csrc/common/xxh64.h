// XXH64 primitives (public-domain algorithm by Y. Collet) shared by host and device code,
// plus the "striped shard hash" used for change detection:
//
//   shard_hash(D, seed):  D (<= shard bytes) is split into 32-byte stripes; stripe s belongs to
//   lane s % 256.  Lane l hashes the concatenation of its stripes (the final stripe of D may
//   be partial) with XXH64(seed).  The shard digest is XXH64(seed) of the 256 lane digests
//   laid out little-endian (2048 bytes).
//
// The striping lets one 256-thread workgroup read a shard fully coalesced while every lane
// runs an independent XXH64; a host reference is `xxhash.xxh64` over the same byte strings.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define TPI_XHD __host__ __device__
#else
#define TPI_XHD
#endif

#define TPI_XXH_P1 11400714785074694791ULL
#define TPI_XXH_P2 14029467366897019727ULL
#define TPI_XXH_P3 1609587929392839161ULL
#define TPI_XXH_P4 9650029242287828579ULL
#define TPI_XXH_P5 2870177450012600261ULL
#define TPI_HASH_LANES 256
#define TPI_HASH_STRIPE 32

TPI_XHD static inline uint64_t tpi_rotl64(uint64_t x, int r) {
  return (x << r) | (x >> (64 - r));
}
TPI_XHD static inline uint64_t tpi_xxh_round(uint64_t acc, uint64_t in) {
  acc += in * TPI_XXH_P2;
  acc = tpi_rotl64(acc, 31);
  return acc * TPI_XXH_P1;
}
TPI_XHD static inline uint64_t tpi_xxh_merge(uint64_t h, uint64_t v) {
  h ^= tpi_xxh_round(0, v);
  return h * TPI_XXH_P1 + TPI_XXH_P4;
}
TPI_XHD static inline uint64_t tpi_xxh_converge(uint64_t v1, uint64_t v2, uint64_t v3,
                                                uint64_t v4) {
  uint64_t h = tpi_rotl64(v1, 1) + tpi_rotl64(v2, 7) + tpi_rotl64(v3, 12) + tpi_rotl64(v4, 18);
  h = tpi_xxh_merge(h, v1);
  h = tpi_xxh_merge(h, v2);
  h = tpi_xxh_merge(h, v3);
  return tpi_xxh_merge(h, v4);
}
TPI_XHD static inline uint64_t tpi_xxh_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= TPI_XXH_P2;
  h ^= h >> 29;
  h *= TPI_XXH_P3;
  h ^= h >> 32;
  return h;
}
// Tail (< 32 bytes) and avalanche; `p` points at the remaining bytes.
TPI_XHD static inline uint64_t tpi_xxh_finish(uint64_t h, const uint8_t* p, uint32_t rem) {
  while (rem >= 8) {
    uint64_t k;
    memcpy(&k, p, 8);
    h ^= tpi_xxh_round(0, k);
    h = tpi_rotl64(h, 27) * TPI_XXH_P1 + TPI_XXH_P4;
    p += 8;
    rem -= 8;
  }
  if (rem >= 4) {
    uint32_t k;
    memcpy(&k, p, 4);
    h ^= (uint64_t)k * TPI_XXH_P1;
    h = tpi_rotl64(h, 23) * TPI_XXH_P2 + TPI_XXH_P3;
    p += 4;
    rem -= 4;
  }
  while (rem) {
    h ^= (uint64_t)(*p) * TPI_XXH_P5;
    h = tpi_rotl64(h, 11) * TPI_XXH_P1;
    ++p;
    --rem;
  }
  return tpi_xxh_avalanche(h);
}

// Plain one-shot XXH64 (host reference and small buffers).
static inline uint64_t tpi_xxh64(const void* data, uint64_t len, uint64_t seed) {
  const uint8_t* p = (const uint8_t*)data;
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + TPI_XXH_P1 + TPI_XXH_P2, v2 = seed + TPI_XXH_P2, v3 = seed,
             v4 = seed - TPI_XXH_P1;
    while (p + 32 <= end) {
      uint64_t w[4];
      memcpy(w, p, 32);
      v1 = tpi_xxh_round(v1, w[0]);
      v2 = tpi_xxh_round(v2, w[1]);
      v3 = tpi_xxh_round(v3, w[2]);
      v4 = tpi_xxh_round(v4, w[3]);
      p += 32;
    }
    h = tpi_xxh_converge(v1, v2, v3, v4);
  } else {
    h = seed + TPI_XXH_P5;
  }
  h += len;
  return tpi_xxh_finish(h, p, (uint32_t)(end - p));
}

// Host reference of the striped shard hash for one shard.
static inline uint64_t tpi_shard_hash_host(const uint8_t* d, uint64_t len, uint64_t seed) {
  uint64_t digests[TPI_HASH_LANES];
  const uint64_t full = len / TPI_HASH_STRIPE;
  const uint32_t rem = (uint32_t)(len % TPI_HASH_STRIPE);
  for (int l = 0; l < TPI_HASH_LANES; ++l) {
    uint64_t nfull = full > (uint64_t)l ? (full - l + TPI_HASH_LANES - 1) / TPI_HASH_LANES : 0;
    int owns_tail = rem && (full % TPI_HASH_LANES) == (uint64_t)l;
    uint64_t mylen = nfull * TPI_HASH_STRIPE + (owns_tail ? rem : 0);
    uint64_t h;
    if (mylen >= 32) {
      uint64_t v1 = seed + TPI_XXH_P1 + TPI_XXH_P2, v2 = seed + TPI_XXH_P2, v3 = seed,
               v4 = seed - TPI_XXH_P1;
      for (uint64_t j = 0; j < nfull; ++j) {
        uint64_t w[4];
        memcpy(w, d + (l + j * TPI_HASH_LANES) * TPI_HASH_STRIPE, 32);
        v1 = tpi_xxh_round(v1, w[0]);
        v2 = tpi_xxh_round(v2, w[1]);
        v3 = tpi_xxh_round(v3, w[2]);
        v4 = tpi_xxh_round(v4, w[3]);
      }
      h = tpi_xxh_converge(v1, v2, v3, v4);
    } else {
      h = seed + TPI_XXH_P5;
    }
    h += mylen;
    digests[l] = tpi_xxh_finish(h, d + full * TPI_HASH_STRIPE, owns_tail ? rem : 0);
  }
  return tpi_xxh64(digests, sizeof(digests), seed);
}
