// Parallel filtered directory copy (the reference's rclone sync.CopyDir, storage.go:158) and
// tree listing for workdir staging.  Files are copied in <= 256 MiB pieces by a thread pool
// with copy_file_range (in-kernel, no user-space bounce), written to "<name>.tpi-partial"
// and renamed once complete; size+mtime equality skips unchanged files (rclone's default
// check), mtimes and permission bits are preserved, empty included directories are created.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "filter.h"

namespace tpi {

struct Entry {
  std::string rel;  // relative path, '/'-separated, no leading '/'
  uint64_t size = 0;
  int64_t mtime_ns = 0;
  uint32_t mode = 0;
  bool is_dir = false;
};

struct TransferStats {
  uint64_t files = 0, bytes = 0, dirs = 0, skipped = 0, skipped_bytes = 0;
  uint64_t cloned = 0;  // files whose extents were shared (reflink) instead of copied
  double seconds = 0;
};

// Walk `root` applying `filter`; returns included files and directories (dirs first in
// pre-order).  Symlinks are skipped (rclone local backend without --links).
std::vector<Entry> walk(const std::string& root, const Filter& filter);

TransferStats copy_dir(const std::string& src, const std::string& dst, const Filter& filter,
                       int threads, uint64_t piece_bytes);

// rm -rf; returns number of entries removed.  Missing path -> 0.
uint64_t remove_tree(const std::string& path);

// Staging reads: read pieces of files into a caller buffer (typically pinned host memory the
// GPU DMA engine reads from) with a thread pool of pread()s.
struct ReadPiece {
  std::string path;
  uint64_t file_off, len, dst_off;
};
uint64_t read_pieces(const std::vector<ReadPiece>& pieces, uint8_t* dst, int threads);
// Inverse for spills: write buffer ranges into files (created/truncated to `size`).
uint64_t write_pieces(const std::vector<ReadPiece>& pieces, const uint8_t* src, int threads);

}  // namespace tpi
