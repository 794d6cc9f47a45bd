// Internals shared by the engine translation units of libtpi_hip.so (engine*.hip): the
// engine and pinner structs, the device-kernel launchers of kernels.hip / codec.hip, and
// the pipelines' common helpers.  Not part of the C ABI (tpi_hip.h is).
#pragma once
#include <errno.h>
#include <signal.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../common/crc32c.h"
#include "../common/tpz.h"
#include "internal.h"
#include "tpi_hip.h"

extern "C" hipError_t tpi_launch_stream_crc(int mode, const tpi_seg* segs, int nseg,
                                            uint64_t stream_base, uint64_t len, void* buf,
                                            uint64_t tile_bytes, const tpi_crc_tables* tables,
                                            uint32_t* crcs, uint32_t init_full,
                                            uint32_t init_last, unsigned long long* bad,
                                            int staged, hipStream_t stream);
extern "C" hipError_t tpi_launch_stream_copy(const tpi_seg* src, const tpi_seg* dst, int nseg,
                                             uint64_t stream_base, uint64_t len,
                                             uint64_t tile_bytes, const tpi_crc_tables* tables,
                                             uint32_t* crcs, uint32_t init_full,
                                             uint32_t init_last, unsigned long long* bad,
                                             hipStream_t stream);
extern "C" hipError_t tpi_launch_transposes(const tpi_seg* host_segs, int nseg, uint64_t base,
                                            uint64_t len, void* buf, int dir,
                                            hipStream_t stream);
extern "C" hipError_t tpi_launch_shard_hash(const void* data, uint64_t nbytes,
                                            uint64_t shard_bytes, uint64_t seed, uint64_t* out,
                                            hipStream_t stream);
extern "C" hipError_t tpi_launch_pack_list(const tpi_seg* segs, int nseg, uint64_t total,
                                           const uint32_t* list, uint32_t n, void* buf,
                                           uint64_t tile_bytes, const tpi_crc_tables* tables,
                                           uint32_t* crcs, uint32_t init_full,
                                           uint32_t init_last, hipStream_t stream);
extern "C" hipError_t tpi_launch_stream_hash(const tpi_seg* segs, int nseg, uint64_t total,
                                             uint64_t tile_bytes, uint64_t seed, uint64_t* out,
                                             hipStream_t stream);
extern "C" hipError_t tpi_launch_dirty_tiles(const uint64_t* hash, uint64_t* prev, uint64_t n,
                                             int all, uint32_t* idx, unsigned int* count,
                                             hipStream_t stream);
extern "C" hipError_t tpi_launch_stream_copy_hash(const tpi_seg* src, const tpi_seg* dst,
                                                  int nseg, uint64_t stream_base, uint64_t len,
                                                  uint64_t total, uint64_t tile_bytes,
                                                  uint64_t seed, uint64_t* digests,
                                                  unsigned long long* bad, hipStream_t stream);

extern "C" hipError_t tpi_launch_tpz_encode(const void* raw, uint64_t len, uint64_t tile,
                                            void* meta, uint32_t* csize, uint32_t* csize_host,
                                            void* out, hipStream_t stream);
extern "C" hipError_t tpi_launch_tpz_decode(const void* comp, const uint64_t* coff,
                                            uint64_t comp_base, uint64_t len, uint64_t tile,
                                            void* raw, hipStream_t stream);

#define TPI_SYNC_SEED 0x7470692d73796e63ull  // "tpi-sync"

// roctx range around each pipeline call: `rocprofv3 --marker-trace` shows save/restore/sync
// phases next to the kernels and copies they issued (no cost when no tool is attached).
struct TpiRange {
  explicit TpiRange(const char* name) { roctxRangePushA(name); }
  ~TpiRange() { roctxRangePop(); }
};

#define HIP_OK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return tpi_fail(std::string(#expr) + ": " + hipGetErrorString(e_));               \
  } while (0)

// Progressive pinning of a (large, existing) host region: a toucher thread faults the pages
// in window by window with a pool of threads, a registrar thread hipHostRegisters each window
// once it is touched.  `ready` = bytes from the base that are registered (a growing prefix),
// so a restore can DMA window k while window k+1 is still being pinned.
struct tpi_pinner {
  uint8_t* base = nullptr;
  uint64_t bytes = 0, window = 0;
  int threads = 8;
  int device = 0;
  std::atomic<uint64_t> touched{0}, ready{0};
  std::atomic<bool> failed{false}, stop{false};
  // held: no window is registered until released (tpi_host_pin_hold) or a copy needs one
  // (wait_pinned): a successor copying its predecessor's HBM keeps the GPU's page-table
  // updates for 100 GB of host pages out of its IPC imports' way
  std::atomic<bool> held{false};
  std::thread toucher, registrar;
  std::vector<uint8_t*> registered;
  std::string error;
};

struct tpi_engine {
  int device = 0;
  uint64_t chunk = 0, tile = 0;
  int nbuf = 0;
  hipStream_t compute = nullptr, copy = nullptr;
  // streamed restore: the per-chunk CRC / blob-offset uploads.  A small host -> device copy
  // does not return before its stream has reached it, so on the copy or compute stream it
  // held the issuing thread -- and the next chunk's H2D -- behind the previous chunk's work.
  hipStream_t aux = nullptr;
  std::vector<hipEvent_t> ev_c;  // aux uploads of staging slot b done
  // streamed restore, behind a save that shares the PCIe link: a chunk's H2D split over the
  // copy stream and this one (HIP gives each stream its own SDMA engine) takes the larger share
  // of a duplex link -- in/out 56/34 GB/s instead of 46/51 (profiles/duplex_split_round3.md)
  hipStream_t copy2 = nullptr;
  std::vector<hipEvent_t> ev_d;  // second half of staging slot b copied
  uint64_t split_lead = 2;       // split once the restore trails the writer by this many chunks
  uint64_t split_chunks = 0;     // chunks split by the last streamed restore
  // staging ring: allocated at the first pipeline that needs it (ensure_staging), so an
  // engine that only runs the HBM hand-off copy -- a parked successor's prewarmed one --
  // holds no staging HBM
  std::vector<void*> staging;
  uint64_t staging_bytes = 0;
  std::vector<hipEvent_t> ev_a, ev_b;  // save: packed/copied; restore: copied/unpacked
  hipEvent_t ev_wait = nullptr, ev_done = nullptr;
  hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;  // timing: the hand-off kernels' device time
  // The HBM hand-off's copy runs on a stream of the device's highest priority
  // (TPI_HANDOFF_PRIORITY=high, default; "normal": on `compute`): during a hot hand-off the
  // predecessor's save (its pack / codec kernels) shares the GPU, and its workgroups then
  // queue behind the copy's instead of interleaving with them.
  hipStream_t urgent = nullptr;
  hipEvent_t ev_prio = nullptr;
  tpi_crc_tables* tables = nullptr;
  tpi_seg* d_segs = nullptr;
  size_t seg_cap = 0;
  uint32_t* d_crcs = nullptr;
  size_t crc_cap = 0;
  unsigned long long* d_bad = nullptr;
  // incremental sync state: digests of the last synced content (valid only until a full
  // save/restore rewrites one side)
  uint64_t* d_hash = nullptr;
  uint64_t* d_prev = nullptr;
  uint32_t* d_idx = nullptr;
  unsigned int* d_count = nullptr;
  size_t hash_cap = 0;
  // HBM hand-off: tile digests of the fused copy, checked by its read-back pass
  uint64_t* d_digest = nullptr;
  size_t digest_cap = 0;
  tpi_seg* d_src = nullptr;  // the hand-off's source descriptors (kept: no hipFree per call)
  size_t src_cap = 0;
  uint64_t hash_ntiles = 0;
  bool hash_valid = false;
  // TPZ1 codec: raw pack scratch (one chunk), per-tile headers of the chunk in flight,
  // blob sizes / offsets of the whole stream
  void* zraw = nullptr;
  void* d_meta = nullptr;
  uint32_t* d_csize = nullptr;
  uint64_t* d_coff = nullptr;
  uint64_t* h_coff = nullptr;  // pinned: per-chunk slices go up asynchronously (restore_stream)
  size_t z_cap = 0;
  // host region registered window by window (tpi_host_pin_start): host copies are split at
  // window boundaries and wait until their window is pinned (tpi_engine_set_host_region)
  const uint8_t* hbase = nullptr;
  uint64_t hbytes = 0, hwin = 0;
  tpi_pinner* pinner = nullptr;
  // D2H on an SDMA engine (sdma.cpp), one lane per staging buffer + one for direct spills;
  // nullptr = hipMemcpyAsync on the copy stream (TPI_D2H_ENGINE=blit, or no engine)
  tpi_sdma* sdma = nullptr;
  // H2D of streamed restores on an SDMA engine of their own (tpi_engine_set_h2d_sdma), host
  // driven like the saves' D2H: off HIP's H2D engine, which the driver's clears of freed HBM
  // share (profiles/round4/materialize_170g.md); nullptr = hipMemcpyAsync
  tpi_sdma* sdma_in = nullptr;
  // streaming hand-off: a save publishes {tiles, stream bytes} already in host memory here
  // (tpi_engine_set_progress); a reader in another process restores behind it
  uint64_t* progress = nullptr;
  std::mutex mu;
};

namespace tpi_engine_detail {

inline int fail(const std::string& what) { return tpi_fail(what); }
const tpi_crc_tables& host_tables();
int device_tables(int dev, tpi_crc_tables** out);
uint32_t init_for(uint64_t len);
int check_segments(const tpi_seg* segs, int n, uint64_t total);
bool extents_disjoint(const tpi_seg* segs, int n);
bool wait_pinned(tpi_pinner* p, uint64_t end);
hipError_t region_copy(tpi_engine* e, void* dst, const void* src, size_t n, hipMemcpyKind kind,
                       hipStream_t s);
bool host_locked(const void* p);
int sdma_region_d2h(tpi_engine* e, int lane, void* dst, const void* src, size_t n);
int sdma_region_h2d(tpi_engine* e, int lane, void* dst, const void* src, size_t n);
int staging_free(tpi_engine* e, int b, hipStream_t producer);
int staging_ready(tpi_engine* e, int b, hipStream_t producer);
int staging_d2h(tpi_engine* e, int b, void* dst, const void* src, size_t n);
int staging_sent(tpi_engine* e, int b);
int drain_d2h(tpi_engine* e);
// Streaming hand-off, save side.  Chunk j's end: first tile after it, stream bytes after it.
struct ChunkMark {
  uint64_t tile_end, byte_end;
};
int publish_chunk(tpi_engine* e, const std::vector<ChunkMark>& marks, uint64_t j,
                  uint64_t* tiles_published, uint32_t* crcs_out);
bool writer_alive(uint64_t pid);
int wait_published(const uint64_t* words, uint64_t tiles, double timeout_s);
// `staging`: the caller's pipeline moves data through the staging ring (ensure_staging)
int prepare(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, bool staging = true);
int ensure_staging(tpi_engine* e);
void* device_view(void* host);
void* meta_view(tpi_engine* e, const void* host, uint64_t bytes, bool restore_side);
int prepare_codec(tpi_engine* e, uint64_t ntiles);

}  // namespace tpi_engine_detail
