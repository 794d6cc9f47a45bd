// Parallel checkpoint file I/O (see fileio.cpp).
#pragma once
#include <stdint.h>

#include <string>

namespace tpi {

// Write [src, src + n) to a new file at `path` with `threads` writers; fsync when `sync`.
// Returns "" or an error text.
std::string write_file(const std::string& path, const void* src, uint64_t n, int threads,
                       bool sync);

// Read [offset, offset + n) of `path` into `dst` chunk by chunk; after each chunk publish
// words[1] = bytes read, words[0] = tiles whose end offset (tile_ends, ascending) is covered
// (words may be null).  Returns "" or an error text.
std::string read_stream(const std::string& path, void* dst, uint64_t offset, uint64_t n,
                        int threads, uint64_t chunk, uint64_t* words, const uint64_t* tile_ends,
                        uint64_t ntiles);

}  // namespace tpi
