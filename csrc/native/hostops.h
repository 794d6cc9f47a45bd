#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../hip/tpi_hip.h"  // tpi_seg (plain C struct shared with the device path)

namespace tpi {

uint32_t crc32c(const void* data, size_t n, uint32_t crc = 0);
uint32_t crc32c_combine(uint32_t a, uint32_t b, uint64_t len_b);
// CRC32C of the whole stream from its per-tile CRCs.
uint32_t crc32c_combine_tiles(const uint32_t* crcs, uint64_t ntiles, uint64_t tile,
                              uint64_t total);
void crc32c_tiles(const void* data, uint64_t n, uint64_t tile, uint32_t* out, int threads);
void shard_hash(const void* data, uint64_t n, uint64_t shard, uint64_t seed, uint64_t* out,
                int threads);
void pack(const tpi_seg* segs, int n, uint64_t total, void* stream, uint64_t tile,
          uint32_t* crcs, int threads);
uint64_t unpack(const tpi_seg* segs, int n, uint64_t total, const void* stream, uint64_t tile,
                const uint32_t* crcs, int threads, int64_t* first_bad);

// Page-cache residency of a file: bytes of its pages in memory (mincore), and whether it
// lives on tmpfs/shmem (whose pages pin slowly for DMA).  Returns -1 if it cannot be mapped.
int64_t resident_bytes(const char* path, uint64_t* size, int* tmpfs);

// TPZ1 codec (csrc/common/tpz.h) over a stream of tiles: blobs are written back to back,
// sizes to `csizes`; returns the compressed length.  Decode returns -1, or the first tile
// whose blob is malformed (that tile is zero-filled).
uint64_t tpz_encode_stream(const void* src, uint64_t total, uint64_t tile, void* dst,
                           uint32_t* csizes, int threads);
int64_t tpz_decode_stream(const void* src, const uint32_t* csizes, uint64_t total, uint64_t tile,
                          void* dst, int threads);

}  // namespace tpi
