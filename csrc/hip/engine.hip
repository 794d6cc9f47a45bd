// Host side of libtpi_hip.so: per-device engine (streams, staging ring, CRC tables), the
// save/restore pipelines and NUMA-local pinned host mappings.
//
// Save (TPI_MODE_SDMA):  for chunk k (buffer b = k % nbuf)
//     compute: wait copied[b] (k >= nbuf) -> pack+CRC kernel into staging[b] -> record packed[b]
//     copy:    wait packed[b] -> hipMemcpyAsync D2H staging[b] -> host + k*chunk -> copied[b]
//   so packing chunk k+1 overlaps the PCIe transfer of chunk k; the copy engine never idles.
// Save (TPI_MODE_DIRECT): one pack kernel streams straight into the host-mapped destination.
// Restore mirrors both (H2D on the copy stream, unpack+verify on the compute stream).
// Save/restore with the TPZ1 codec (tpi_save_z / tpi_restore_z): pack+CRC into a raw scratch
// chunk, byte-plane encode into staging[b], D2H only the compressed bytes (and the inverse).
// Incremental sync (tpi_sync): per-tile digests from the tensors, pack + D2H of dirty tiles.
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

namespace {

thread_local std::string g_err;

// roctx range around each pipeline call: `rocprofv3 --marker-trace` shows save/restore/sync
// phases next to the kernels and copies they issued (no cost when no tool is attached).
struct Range {
  explicit Range(const char* name) { roctxRangePushA(name); }
  ~Range() { roctxRangePop(); }
};

int fail(const std::string& what) {
  g_err = what;
  return -1;
}

#define HIP_OK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(std::string(#expr) + ": " + hipGetErrorString(e_));                   \
  } while (0)

const tpi_crc_tables& host_tables() {
  static tpi_crc_tables t;
  static std::once_flag once;
  std::call_once(once, [] { tpi_crc_tables_init(&t); });
  return t;
}

// Device copies of the CRC tables, one per device (lazily created, never freed).  The
// bank-column layout (TPI_CRC_COLS_WORDS dwords, tpi_crc_cols_init) follows the struct in
// the same allocation: the CRC-only kernel reads it at `tables + 1`.
std::mutex g_tab_mu;
std::vector<tpi_crc_tables*> g_dev_tables;

int device_tables(int dev, tpi_crc_tables** out) {
  std::lock_guard<std::mutex> lk(g_tab_mu);
  if ((int)g_dev_tables.size() <= dev) g_dev_tables.resize(dev + 1, nullptr);
  if (!g_dev_tables[dev]) {
    static_assert(sizeof(tpi_crc_tables) % 16 == 0, "column tables must stay 16-B aligned");
    std::vector<uint8_t> img(sizeof(tpi_crc_tables) + TPI_CRC_COLS_WORDS * 4);
    memcpy(img.data(), &host_tables(), sizeof(tpi_crc_tables));
    tpi_crc_cols_init(&host_tables(), (uint32_t*)(img.data() + sizeof(tpi_crc_tables)));
    tpi_crc_tables* d = nullptr;
    HIP_OK(hipMalloc(&d, img.size()));
    HIP_OK(hipMemcpy(d, img.data(), img.size(), hipMemcpyHostToDevice));
    g_dev_tables[dev] = d;
  }
  *out = g_dev_tables[dev];
  return 0;
}

uint32_t init_for(uint64_t len) {
  return tpi_multmodp(tpi_x8nmodp(len, host_tables().x2n), 0xFFFFFFFFu);
}

int check_segments(const tpi_seg* segs, int n, uint64_t total) {
  if (n <= 0) return fail("no segments");
  if (segs[0].off != 0) return fail("first segment must start at offset 0");
  for (int i = 0; i < n; ++i) {
    if (segs[i].off % 16) return fail("segment offset not 16-byte aligned");
    if (i && segs[i].off < segs[i - 1].off + segs[i - 1].nbytes)
      return fail("segments overlap or are unsorted");
    if (segs[i].off + segs[i].nbytes > total) return fail("segment exceeds stream");
    if (segs[i].kind > TPI_SEG_TRANSPOSE) return fail("unknown segment kind");
    if (segs[i].kind != TPI_SEG_CONTIG && (segs[i].elem == 0 || segs[i].ndim < 1 ||
                                           segs[i].ndim > TPI_MAX_DIMS))
      return fail("bad strided segment descriptor");
    if (segs[i].kind == TPI_SEG_TRANSPOSE &&
        (segs[i].ndim < 2 || segs[i].ndim > 3 || segs[i].elem > 8 ||
         (segs[i].elem & (segs[i].elem - 1)) || segs[i].ptr % segs[i].elem ||
         segs[i].strides[segs[i].ndim - 2] != 1))
      return fail("bad transpose segment descriptor");
  }
  if (total % 16) return fail("stream length must be a multiple of 16");
  return 0;
}

// Do the destination segments occupy disjoint memory?  Extent of a strided segment: from its
// lowest to its highest element (negative strides included), so interleaved views of one
// storage count as overlapping -- conservative, which only costs them the inline check.
bool extents_disjoint(const tpi_seg* segs, int n) {
  std::vector<std::pair<uint64_t, uint64_t>> ext;
  ext.reserve((size_t)n);
  for (int i = 0; i < n; ++i) {
    if (segs[i].nbytes == 0) continue;
    uint64_t lo = segs[i].ptr, hi = segs[i].ptr + segs[i].nbytes;
    if (segs[i].kind != TPI_SEG_CONTIG) {
      int64_t neg = 0, pos = 0;
      for (int d = 0; d < segs[i].ndim && d < TPI_MAX_DIMS; ++d) {
        const int64_t span = (segs[i].sizes[d] - 1) * segs[i].strides[d] * (int64_t)segs[i].elem;
        (span < 0 ? neg : pos) += span;
      }
      lo = segs[i].ptr + neg;  // neg <= 0
      hi = segs[i].ptr + pos + segs[i].elem;
    }
    ext.push_back({lo, hi});
  }
  std::sort(ext.begin(), ext.end());
  for (size_t i = 1; i < ext.size(); ++i)
    if (ext[i].first < ext[i - 1].second) return false;
  return true;
}

}  // namespace

// Error reporting for the other translation units of the library (internal.h).
int tpi_fail(const std::string& what) { return fail(what); }

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
  std::vector<void*> staging;
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


namespace {

// Wait until the pinner has registered `end` bytes of the region (false: pinning failed).
bool wait_pinned(tpi_pinner* p, uint64_t end) {
  p->held.store(false, std::memory_order_release);  // a copy needs the region: pin it now
  while (p->ready.load(std::memory_order_acquire) < end) {
    if (p->failed.load()) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  return true;
}

// hipMemcpyAsync for the engine's pipelines: a host side inside a window-registered region is
// split at window boundaries (one registration per window) and waits for its window.
hipError_t region_copy(tpi_engine* e, void* dst, const void* src, size_t n, hipMemcpyKind kind,
                       hipStream_t s) {
  const uint8_t* h = (const uint8_t*)(kind == hipMemcpyHostToDevice ? src : dst);
  if (!e->hwin || kind == hipMemcpyDeviceToDevice || h < e->hbase || h >= e->hbase + e->hbytes)
    return hipMemcpyAsync(dst, src, n, kind, s);
  uint64_t off = (uint64_t)(h - e->hbase), done = 0;
  while (done < n) {
    const uint64_t at = off + done;
    const uint64_t len = std::min<uint64_t>(n - done, (at / e->hwin + 1) * e->hwin - at);
    if (e->pinner && !wait_pinned(e->pinner, std::min(e->hbytes, at + len)))
      return hipErrorInvalidValue;
    hipError_t err =
        hipMemcpyAsync((uint8_t*)dst + done, (const uint8_t*)src + done, len, kind, s);
    if (err != hipSuccess) return err;
    done += len;
  }
  return hipSuccess;
}

// An SDMA engine can only reach host pages locked for the GPU; anything else (pageable
// memory) would fault, so it takes HIP's staged path instead.
bool host_locked(const void* p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // not a HIP pointer: leave no error for the next caller to see
    return false;
  }
  return at.type == hipMemoryTypeHost && at.devicePointer != nullptr;
}

// D2H of one piece on SDMA lane `lane`, split at pinned-window boundaries like region_copy.
// The producer of `src` has completed (the caller synchronised on its event).
int sdma_region_d2h(tpi_engine* e, int lane, void* dst, const void* src, size_t n) {
  const uint8_t* h = (const uint8_t*)dst;
  if (!e->hwin || h < e->hbase || h >= e->hbase + e->hbytes) {
    if (!host_locked(dst)) {
      HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, e->copy));
      HIP_OK(hipStreamSynchronize(e->copy));
      return 0;
    }
    return tpi_sdma_d2h(e->sdma, lane, dst, src, n);
  }
  uint64_t off = (uint64_t)(h - e->hbase), done = 0;
  while (done < n) {
    const uint64_t at = off + done;
    const uint64_t len = std::min<uint64_t>(n - done, (at / e->hwin + 1) * e->hwin - at);
    if (e->pinner && !wait_pinned(e->pinner, std::min(e->hbytes, at + len)))
      return fail("host region pinning failed");
    if (tpi_sdma_d2h(e->sdma, lane, (uint8_t*)dst + done, (const uint8_t*)src + done, len))
      return -1;
    done += len;
  }
  return 0;
}

// H2D of one piece on the restore's SDMA lane `lane`, split at pinned-window boundaries.
int sdma_region_h2d(tpi_engine* e, int lane, void* dst, const void* src, size_t n) {
  const uint8_t* h = (const uint8_t*)src;
  if (!e->hwin || h < e->hbase || h >= e->hbase + e->hbytes)
    return tpi_sdma_h2d(e->sdma_in, lane, dst, src, n);
  uint64_t off = (uint64_t)(h - e->hbase), done = 0;
  while (done < n) {
    const uint64_t at = off + done;
    const uint64_t len = std::min<uint64_t>(n - done, (at / e->hwin + 1) * e->hwin - at);
    if (e->pinner && !wait_pinned(e->pinner, std::min(e->hbytes, at + len)))
      return fail("host region pinning failed");
    if (tpi_sdma_h2d(e->sdma_in, lane, (uint8_t*)dst + done, h + done, len)) return -1;
    done += len;
  }
  return 0;
}

// The pipelines' D2H legs.  Staging buffer b is free again once its copies are done:
//   blit: the copy stream records copied[b]; the producer stream waits for it.
//   SDMA: the copies of buffer b are signalled on lane b; the host waits for the lane before
//         the producer writes the buffer again, and issues a copy once the producer's event
//         (packed[b]) has completed.
int staging_free(tpi_engine* e, int b, hipStream_t producer) {
  if (e->sdma) return tpi_sdma_wait(e->sdma, b);
  HIP_OK(hipStreamWaitEvent(producer, e->ev_b[b], 0));
  return 0;
}

// Make the producer's work up to now (recorded as packed[b]) the precondition of the copies
// that follow for buffer b.
int staging_ready(tpi_engine* e, int b, hipStream_t producer) {
  HIP_OK(hipEventRecord(e->ev_a[b], producer));
  if (e->sdma) {
    HIP_OK(hipEventSynchronize(e->ev_a[b]));
  } else {
    HIP_OK(hipStreamWaitEvent(e->copy, e->ev_a[b], 0));
  }
  return 0;
}

int staging_d2h(tpi_engine* e, int b, void* dst, const void* src, size_t n) {
  if (e->sdma) return sdma_region_d2h(e, b, dst, src, n);
  HIP_OK(region_copy(e, dst, src, n, hipMemcpyDeviceToHost, e->copy));
  return 0;
}

int staging_sent(tpi_engine* e, int b) {
  if (!e->sdma) HIP_OK(hipEventRecord(e->ev_b[b], e->copy));
  return 0;
}

int drain_d2h(tpi_engine* e) {
  if (e->sdma && tpi_sdma_wait_all(e->sdma)) return -1;
  HIP_OK(hipStreamSynchronize(e->copy));
  return 0;
}

// Streaming hand-off, save side.  Chunk j's end: first tile after it, stream bytes after it.
struct ChunkMark {
  uint64_t tile_end, byte_end;
};

// Publish that chunks [0, j] are in host memory: wait for chunk j's D2H (its lane, or its
// copied event), copy the tile CRCs it completed to the host, then release-store the
// progress words (bytes first, tiles last: a reader acquires tiles, then reads bytes).
int publish_chunk(tpi_engine* e, const std::vector<ChunkMark>& marks, uint64_t j,
                  uint64_t* tiles_published, uint32_t* crcs_out) {
  const int b = (int)(j % (uint64_t)e->nbuf);
  if (e->sdma) {
    if (tpi_sdma_wait(e->sdma, b)) return -1;
  } else {
    HIP_OK(hipEventSynchronize(e->ev_b[b]));
  }
  const uint64_t t_end = marks[j].tile_end;
  if (t_end > *tiles_published) {
    if (crcs_out)  // else the kernels stored the CRCs in host memory themselves (meta_view)
      HIP_OK(hipMemcpy(crcs_out + *tiles_published, e->d_crcs + *tiles_published,
                       (t_end - *tiles_published) * sizeof(uint32_t), hipMemcpyDeviceToHost));
    *tiles_published = t_end;
  }
  __atomic_store_n(&e->progress[1], marks[j].byte_end, __ATOMIC_RELEASE);
  __atomic_store_n(&e->progress[0], t_end, __ATOMIC_RELEASE);
  return 0;
}

// Streaming hand-off, restore side: block until the writer has published `tiles` tiles.
// Fails when the writer reports failure (words[2] == 3, the progress block's state word) or
// makes no progress for `timeout_s` (it died).
// Is the process that publishes a streamed save (progress word 3) still running?  Zombies
// count as gone: a SIGKILLed predecessor is not reaped at once.
bool writer_alive(uint64_t pid) {
  if (pid == 0 || pid == (uint64_t)getpid()) return true;
  if (kill((pid_t)pid, 0) != 0 && errno == ESRCH) return false;
  char path[64];
  snprintf(path, sizeof(path), "/proc/%llu/stat", (unsigned long long)pid);
  FILE* f = fopen(path, "r");
  if (!f) return true;  // no /proc: trust kill()
  char buf[512];
  const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* rp = strrchr(buf, ')');
  return !(rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X'));
}

int wait_published(const uint64_t* words, uint64_t tiles, double timeout_s) {
  uint64_t seen = __atomic_load_n(&words[0], __ATOMIC_ACQUIRE);
  auto last = std::chrono::steady_clock::now();
  auto last_check = last;
  while (seen < tiles) {
    if (__atomic_load_n(&words[2], __ATOMIC_ACQUIRE) == 3)  // the writer reported a failure
      return fail("the streamed checkpoint failed in its writer");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
    const auto now = std::chrono::steady_clock::now();
    if (std::chrono::duration<double>(now - last_check).count() > 0.02) {
      last_check = now;
      if (__atomic_load_n(&words[0], __ATOMIC_ACQUIRE) < tiles &&
          __atomic_load_n(&words[2], __ATOMIC_ACQUIRE) != 2 &&
          !writer_alive(__atomic_load_n(&words[3], __ATOMIC_ACQUIRE)))
        return fail("the streamed checkpoint's writer exited before finishing it");
    }
    const uint64_t now_tiles = __atomic_load_n(&words[0], __ATOMIC_ACQUIRE);
    if (now_tiles != seen) {
      seen = now_tiles;
      last = std::chrono::steady_clock::now();
    } else if (std::chrono::duration<double>(std::chrono::steady_clock::now() - last).count() >
               timeout_s) {
      return fail("streamed checkpoint stalled at tile " + std::to_string(seen) + " of " +
                  std::to_string(tiles) + " (writer gone?)");
    }
  }
  return 0;
}

}  // namespace

extern "C" {

const char* tpi_last_error(void) { return g_err.c_str(); }
#ifndef TPI_VERSION_STRING
#define TPI_VERSION_STRING "0.0.0-dev"
#endif
int tpi_version(void) { return TPI_ABI_VERSION; }
const char* tpi_version_string(void) { return TPI_VERSION_STRING; }

int tpi_device_count(int* count) {
  HIP_OK(hipGetDeviceCount(count));
  return 0;
}

int tpi_device_pci_bus_id(int device, char* buf, int len) {
  HIP_OK(hipDeviceGetPCIBusId(buf, len, device));
  return 0;
}

int tpi_device_numa_node(int device, int* node) {
  char bus[64] = {0};
  *node = -1;
  if (tpi_device_pci_bus_id(device, bus, sizeof(bus))) return -1;
  for (char* p = bus; *p; ++p) *p = (char)tolower(*p);
  std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return 0;  // unknown topology: no binding
  if (fscanf(f, "%d", node) != 1) *node = -1;
  fclose(f);
  return 0;
}

tpi_engine* tpi_engine_create(int device, uint64_t chunk_bytes, int nbuf, uint64_t tile_bytes) {
  if (tile_bytes == 0 || tile_bytes % TPI_ROW_BYTES) {
    fail("tile_bytes must be a positive multiple of 4096");
    return nullptr;
  }
  if (chunk_bytes < tile_bytes) chunk_bytes = tile_bytes;
  chunk_bytes -= chunk_bytes % tile_bytes;
  if (nbuf < 1) nbuf = 1;
  tpi_engine* e = new tpi_engine();
  e->device = device;
  e->chunk = chunk_bytes;
  e->tile = tile_bytes;
  e->nbuf = nbuf;
  auto bail = [&](const char* what, hipError_t err) -> tpi_engine* {
    fail(std::string(what) + ": " + hipGetErrorString(err));
    tpi_engine_destroy(e);
    return nullptr;
  };
  hipError_t err;
  // TPI_ENGINE_TRACE=1: the time of each creation step on stderr
  const bool trace = getenv("TPI_ENGINE_TRACE") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto step = [&](const char* what) {
    if (!trace) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "tpi_engine_create: %s %.3f ms\n", what,
            std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  if ((err = hipSetDevice(device)) != hipSuccess) return bail("hipSetDevice", err);
  step("hipSetDevice");
  if ((err = hipStreamCreateWithFlags(&e->compute, hipStreamNonBlocking)) != hipSuccess)
    return bail("hipStreamCreate(compute)", err);
  // the process's first hardware queue: ~137 ms of a cold successor's engine creation, the
  // other streams ~5 ms each (profiles/round5/r5z/engine_create_trace.txt)
  step("compute stream");
  if ((err = hipStreamCreateWithFlags(&e->copy, hipStreamNonBlocking)) != hipSuccess)
    return bail("hipStreamCreate(copy)", err);
  if ((err = hipStreamCreateWithFlags(&e->aux, hipStreamNonBlocking)) != hipSuccess)
    return bail("hipStreamCreate(aux)", err);
  if ((err = hipStreamCreateWithFlags(&e->copy2, hipStreamNonBlocking)) != hipSuccess)
    return bail("hipStreamCreate(copy2)", err);
  step("3 more streams");
  if (const char* lead = getenv("TPI_H2D_SPLIT_LEAD")) {  // "off": never split
    char* end = nullptr;
    const unsigned long long v = strtoull(lead, &end, 10);
    if (strcmp(lead, "off") == 0) e->split_lead = ~0ull;
    else if (end != lead && *end == '\0') e->split_lead = v;  // else: keep the default
  }
  // staging chunks also hold TPZ1 blobs: worst case tpz_bound() per tile
  const uint64_t staging_bytes = chunk_bytes + (chunk_bytes / tile_bytes) * (TPZ_HDR + 128);
  e->staging.assign(nbuf, nullptr);
  e->ev_a.assign(nbuf, nullptr);
  e->ev_b.assign(nbuf, nullptr);
  e->ev_c.assign(nbuf, nullptr);
  e->ev_d.assign(nbuf, nullptr);
  for (int i = 0; i < nbuf; ++i) {
    if ((err = hipEventCreateWithFlags(&e->ev_c[i], hipEventDisableTiming)) != hipSuccess)
      return bail("hipEventCreate", err);
    if ((err = hipEventCreateWithFlags(&e->ev_d[i], hipEventDisableTiming)) != hipSuccess)
      return bail("hipEventCreate", err);
    if ((err = hipMalloc(&e->staging[i], staging_bytes)) != hipSuccess)
      return bail("hipMalloc(staging)", err);
    if ((err = hipEventCreateWithFlags(&e->ev_a[i], hipEventDisableTiming)) != hipSuccess)
      return bail("hipEventCreate", err);
    if ((err = hipEventCreateWithFlags(&e->ev_b[i], hipEventDisableTiming)) != hipSuccess)
      return bail("hipEventCreate", err);
  }
  step("staging + events");
  if ((err = hipEventCreateWithFlags(&e->ev_wait, hipEventDisableTiming)) != hipSuccess)
    return bail("hipEventCreate", err);
  if ((err = hipEventCreateWithFlags(&e->ev_done, hipEventDisableTiming)) != hipSuccess)
    return bail("hipEventCreate", err);
  if ((err = hipEventCreate(&e->ev_t0)) != hipSuccess || (err = hipEventCreate(&e->ev_t1)) != hipSuccess)
    return bail("hipEventCreate", err);
  {
    const char* prio = getenv("TPI_HANDOFF_PRIORITY");
    if (!prio || strcmp(prio, "normal") != 0) {
      int least = 0, greatest = 0;  // no priority stream: the copy stays on `compute`
      if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
          hipStreamCreateWithPriority(&e->urgent, hipStreamNonBlocking, greatest) != hipSuccess ||
          hipEventCreateWithFlags(&e->ev_prio, hipEventDisableTiming) != hipSuccess) {
        if (e->urgent) (void)hipStreamDestroy(e->urgent);
        e->urgent = nullptr;
      }
    }
  }
  step("events + priority stream");
  if ((err = hipMalloc(&e->d_bad, 2 * sizeof(unsigned long long))) != hipSuccess)
    return bail("hipMalloc(bad)", err);
  if (device_tables(device, &e->tables)) {
    tpi_engine_destroy(e);
    return nullptr;
  }
  step("crc tables");
  e->sdma = tpi_sdma_open(device, nbuf + 1);
  step("sdma lanes");
  return e;
}

void tpi_engine_destroy(tpi_engine* e) {
  if (!e) return;
  // Teardown is best effort: errors here have nowhere useful to go.
  (void)hipSetDevice(e->device);
  if (e->compute) (void)hipStreamSynchronize(e->compute);
  if (e->copy) (void)hipStreamSynchronize(e->copy);
  if (e->aux) (void)hipStreamSynchronize(e->aux);
  if (e->copy2) (void)hipStreamSynchronize(e->copy2);
  tpi_sdma_close(e->sdma);  // waits for copies still in flight
  tpi_sdma_close(e->sdma_in);
  for (void* p : e->staging)
    if (p) (void)hipFree(p);
  for (hipEvent_t ev : e->ev_a)
    if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->ev_b)
    if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->ev_c)
    if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->ev_d)
    if (ev) (void)hipEventDestroy(ev);
  if (e->ev_wait) (void)hipEventDestroy(e->ev_wait);
  if (e->ev_done) (void)hipEventDestroy(e->ev_done);
  if (e->ev_t0) (void)hipEventDestroy(e->ev_t0);
  if (e->ev_t1) (void)hipEventDestroy(e->ev_t1);
  if (e->d_segs) (void)hipFree(e->d_segs);
  if (e->d_crcs) (void)hipFree(e->d_crcs);
  if (e->d_bad) (void)hipFree(e->d_bad);
  if (e->d_hash) (void)hipFree(e->d_hash);
  if (e->d_digest) (void)hipFree(e->d_digest);
  if (e->d_src) (void)hipFree(e->d_src);
  if (e->d_prev) (void)hipFree(e->d_prev);
  if (e->d_idx) (void)hipFree(e->d_idx);
  if (e->d_count) (void)hipFree(e->d_count);
  for (void* p : {e->zraw, e->d_meta, (void*)e->d_csize, (void*)e->d_coff})
    if (p) (void)hipFree(p);
  if (e->h_coff) (void)hipHostFree(e->h_coff);
  if (e->urgent) (void)hipStreamDestroy(e->urgent);
  if (e->ev_prio) (void)hipEventDestroy(e->ev_prio);
  if (e->compute) (void)hipStreamDestroy(e->compute);
  if (e->copy) (void)hipStreamDestroy(e->copy);
  if (e->aux) (void)hipStreamDestroy(e->aux);
  if (e->copy2) (void)hipStreamDestroy(e->copy2);
  delete e;
}

uint64_t tpi_engine_tile_bytes(const tpi_engine* e) { return e->tile; }
uint64_t tpi_engine_chunk_bytes(const tpi_engine* e) { return e->chunk; }
uint32_t tpi_engine_d2h_engine(const tpi_engine* e) { return tpi_sdma_engine(e->sdma); }
uint64_t tpi_engine_split_chunks(const tpi_engine* e) { return e->split_chunks; }

}  // extern "C"

namespace {

int prepare(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total) {
  if (check_segments(segs, n, total)) return -1;
  HIP_OK(hipSetDevice(e->device));
  // a previous call that failed half-way may have left copies out of a staging buffer
  if (e->sdma && tpi_sdma_wait_all(e->sdma)) return -1;
  if ((size_t)n > e->seg_cap) {
    if (e->d_segs) HIP_OK(hipFree(e->d_segs));
    e->seg_cap = std::max<size_t>(n, 64);
    HIP_OK(hipMalloc(&e->d_segs, e->seg_cap * sizeof(tpi_seg)));
  }
  const size_t ntiles = (total + e->tile - 1) / e->tile;
  if (ntiles > e->crc_cap) {
    if (e->d_crcs) HIP_OK(hipFree(e->d_crcs));
    e->crc_cap = std::max<size_t>(ntiles, 1024);
    HIP_OK(hipMalloc(&e->d_crcs, e->crc_cap * sizeof(uint32_t)));
  }
  // Descriptors are tiny; a synchronous copy keeps the host array's lifetime simple.
  HIP_OK(region_copy(e, e->d_segs, segs, n * sizeof(tpi_seg), hipMemcpyHostToDevice,
                        e->compute));
  return 0;
}

void* device_view(void* host) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) return host;
  return d;
}

// Streamed saves and restores keep per-tile metadata (CRCs, blob sizes, blob offsets) where
// the other side reads it -- the kernels store it straight into registered host memory and
// load it from there (sysmem.h) -- instead of one small copy per chunk in each direction.
// Those copies ran as HIP blit kernels on a queue of their own, the only work in flight during
// the ~3 ms stalls of both pipelines traced in profiles/hw_queues_round3.md.  Returns the
// device address of `bytes` at `host`, or nullptr when the kernels cannot reach it (not
// registered, split over two registration windows) or TPI_DIRECT_META=0: then the copies.
// TPI_DIRECT_META: "save" (default) the saves only, "1" both sides, "restore" the restores
// only, "0" none.  Measured with bench.py on MI355X (profiles/round4/direct_meta.md): saves
// +1.4 % (no synchronous CRC copy at publish, no blob-size copy per chunk); restores reading
// CRCs and blob offsets over PCIe from their kernels -0.5 to -1 %, so they keep the copies.
void* meta_view(tpi_engine* e, const void* host, uint64_t bytes, bool restore_side) {
  static const int sides = [] {  // bit 0: saves, bit 1: restores
    const char* v = getenv("TPI_DIRECT_META");
    if (!v || !strcmp(v, "save")) return 1;
    if (!strcmp(v, "0") || !strcmp(v, "false") || !strcmp(v, "no")) return 0;
    if (!strcmp(v, "restore")) return 2;
    return 3;
  }();
  if (!(sides & (restore_side ? 2 : 1)) || !host || !bytes) return nullptr;
  const uint8_t* h = (const uint8_t*)host;
  if (e->hwin && h >= e->hbase && h < e->hbase + e->hbytes) {
    const uint64_t at = (uint64_t)(h - e->hbase);
    if (at / e->hwin != (at + bytes - 1) / e->hwin) return nullptr;
    if (e->pinner && !wait_pinned(e->pinner, std::min(e->hbytes, at + bytes))) return nullptr;
  }
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void*>(host), 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
}

}  // namespace

extern "C" {

int tpi_save(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* host_dst,
             uint32_t* crcs_out, int mode, uint64_t wait_stream, tpi_stats* stats) {
  Range range("tpi_save");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  if (prepare(e, segs, n, total)) return -1;
  e->hash_valid = false;  // host content no longer matches the last sync's digests
  if (wait_stream != TPI_NO_STREAM) {
    HIP_OK(hipEventRecord(e->ev_wait, (hipStream_t)wait_stream));
    HIP_OK(hipStreamWaitEvent(e->compute, e->ev_wait, 0));
  }
  const uint64_t tile = e->tile;
  const uint32_t init_full = init_for(tile);
  const uint32_t init_last = init_for(total % tile ? total % tile : tile);
  uint64_t nchunks = 0;
  bool direct_crcs = false;
  if (mode == TPI_MODE_DIRECT) {
    HIP_OK(tpi_launch_stream_crc(0, e->d_segs, n, 0, total, device_view(host_dst), tile,
                                 e->tables, e->d_crcs, init_full, init_last, nullptr, 0,
                                 e->compute));
    nchunks = 1;
  } else {
    uint8_t* dst = (uint8_t*)host_dst;
    std::vector<ChunkMark> marks;
    uint64_t published = 0;
    // streamed: the CRC kernel stores each tile's CRC in crcs_out itself (meta_view)
    uint32_t* crc_host =
        e->progress ? (uint32_t*)meta_view(e, crcs_out, (total + tile - 1) / tile *
                                                            sizeof(uint32_t), false)
                    : nullptr;
    uint32_t* crc_dst = crc_host ? crc_host : e->d_crcs;
    for (uint64_t base = 0, k = 0; base < total; base += e->chunk, ++k) {
      const int b = (int)(k % e->nbuf);
      const uint64_t len = std::min(e->chunk, total - base);
      if (k >= (uint64_t)e->nbuf && staging_free(e, b, e->compute)) return -1;
      HIP_OK(tpi_launch_transposes(segs, n, base, len, e->staging[b], 0, e->compute));
      HIP_OK(tpi_launch_stream_crc(0, e->d_segs, n, base, len, e->staging[b], tile, e->tables,
                                   crc_dst, init_full, init_last, nullptr, 1, e->compute));
      if (staging_ready(e, b, e->compute) || staging_d2h(e, b, dst + base, e->staging[b], len) ||
          staging_sent(e, b))
        return -1;
      marks.push_back({(base + len + tile - 1) / tile, base + len});
      // chunk k is queued behind chunk k-1 on the engine: publishing k-1 keeps it busy
      if (e->progress && k >= 1 &&
          publish_chunk(e, marks, k - 1, &published, crc_host ? nullptr : crcs_out))
        return -1;
      nchunks = k + 1;
    }
    if (e->progress && !marks.empty() &&
        publish_chunk(e, marks, marks.size() - 1, &published, crc_host ? nullptr : crcs_out))
      return -1;
    if (crc_host) direct_crcs = true;
  }
  const uint64_t ntiles = (total + tile - 1) / tile;
  if (!direct_crcs)
    HIP_OK(region_copy(e, crcs_out, e->d_crcs, ntiles * sizeof(uint32_t), hipMemcpyDeviceToHost,
                       e->compute));
  if (drain_d2h(e)) return -1;
  HIP_OK(hipStreamSynchronize(e->compute));
  if (stats) {
    stats->copy_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats->pack_ms = 0;
    stats->bytes = total;
    stats->chunks = nchunks;
  }
  return 0;
}

int tpi_restore(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, const void* host_src,
                const uint32_t* crcs, int mode, uint64_t signal_stream, uint64_t* bad_tiles,
                int64_t* first_bad, tpi_stats* stats) {
  Range range("tpi_restore");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  if (prepare(e, segs, n, total)) return -1;
  e->hash_valid = false;  // tensors are overwritten: digests of the last sync are stale
  const uint64_t tile = e->tile;
  const uint64_t ntiles = (total + tile - 1) / tile;
  const uint32_t init_full = init_for(tile);
  const uint32_t init_last = init_for(total % tile ? total % tile : tile);
  unsigned long long bad_init[2] = {0ull, ~0ull};
  if (signal_stream != TPI_NO_STREAM) {
    // The unpack overwrites the caller's tensors: order it after the caller's pending work
    // on them (e.g. a zero_() still queued on torch's stream).
    HIP_OK(hipEventRecord(e->ev_wait, (hipStream_t)signal_stream));
    HIP_OK(hipStreamWaitEvent(e->compute, e->ev_wait, 0));
  }
  HIP_OK(region_copy(e, e->d_crcs, crcs, ntiles * sizeof(uint32_t), hipMemcpyHostToDevice,
                        e->compute));
  HIP_OK(region_copy(e, e->d_bad, bad_init, sizeof(bad_init), hipMemcpyHostToDevice,
                        e->compute));
  uint64_t nchunks = 0;
  if (mode == TPI_MODE_DIRECT) {
    HIP_OK(tpi_launch_stream_crc(1, e->d_segs, n, 0, total, device_view((void*)host_src), tile,
                                 e->tables, e->d_crcs, init_full, init_last, e->d_bad, 0,
                                 e->compute));
    nchunks = 1;
  } else {
    // The copy stream must not start before the CRC/bad uploads are ordered on compute.
    HIP_OK(hipEventRecord(e->ev_wait, e->compute));
    HIP_OK(hipStreamWaitEvent(e->copy, e->ev_wait, 0));
    const uint8_t* src = (const uint8_t*)host_src;
    for (uint64_t base = 0, k = 0; base < total; base += e->chunk, ++k) {
      const int b = (int)(k % e->nbuf);
      const uint64_t len = std::min(e->chunk, total - base);
      if (k >= (uint64_t)e->nbuf) HIP_OK(hipStreamWaitEvent(e->copy, e->ev_b[b], 0));
      HIP_OK(region_copy(e, e->staging[b], src + base, len, hipMemcpyHostToDevice, e->copy));
      HIP_OK(hipEventRecord(e->ev_a[b], e->copy));
      HIP_OK(hipStreamWaitEvent(e->compute, e->ev_a[b], 0));
      HIP_OK(tpi_launch_stream_crc(1, e->d_segs, n, base, len, e->staging[b], tile, e->tables,
                                   e->d_crcs, init_full, init_last, e->d_bad, 1, e->compute));
      HIP_OK(tpi_launch_transposes(segs, n, base, len, e->staging[b], 1, e->compute));
      HIP_OK(hipEventRecord(e->ev_b[b], e->compute));
      nchunks = k + 1;
    }
  }
  unsigned long long bad[2];
  HIP_OK(region_copy(e, bad, e->d_bad, sizeof(bad), hipMemcpyDeviceToHost, e->compute));
  HIP_OK(hipEventRecord(e->ev_done, e->compute));
  if (signal_stream != TPI_NO_STREAM) HIP_OK(hipStreamWaitEvent((hipStream_t)signal_stream, e->ev_done, 0));
  HIP_OK(hipStreamSynchronize(e->compute));
  HIP_OK(hipStreamSynchronize(e->copy));
  HIP_OK(hipStreamSynchronize(e->copy2));
  *bad_tiles = bad[0];
  *first_bad = bad[0] ? (int64_t)bad[1] : -1;
  if (stats) {
    stats->copy_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats->pack_ms = 0;
    stats->bytes = total;
    stats->chunks = nchunks;
  }
  return 0;
}

int tpi_sync(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* host_dst,
             uint32_t* crcs_inout, uint64_t* dev_prev, int full, uint64_t wait_stream,
             uint64_t* dirty_tiles, tpi_stats* stats) {
  Range range("tpi_sync");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  // d_prev is overwritten with the new digests before the dirty tiles reach the host: until
  // this call succeeds, the digests describe content the host may not have.
  const bool was_valid = e->hash_valid;
  e->hash_valid = false;
  if (prepare(e, segs, n, total)) return -1;
  const uint64_t tile = e->tile;
  const uint64_t ntiles = (total + tile - 1) / tile;
  bool valid = was_valid;
  if (ntiles > e->hash_cap) {
    for (void* p : {(void*)e->d_hash, (void*)e->d_prev, (void*)e->d_idx})
      if (p) HIP_OK(hipFree(p));
    e->hash_cap = std::max<size_t>(ntiles, 1024);
    HIP_OK(hipMalloc(&e->d_hash, e->hash_cap * sizeof(uint64_t)));
    HIP_OK(hipMalloc(&e->d_prev, e->hash_cap * sizeof(uint64_t)));
    HIP_OK(hipMalloc(&e->d_idx, e->hash_cap * sizeof(uint32_t)));
    valid = false;
  }
  if (!e->d_count) HIP_OK(hipMalloc(&e->d_count, sizeof(unsigned int)));
  if (e->hash_ntiles != ntiles) valid = false;
  // Caller-owned digests (one array per host slot, Checkpointer slots=2): the caller knows
  // whether they describe the destination's content and says so with `full`.
  uint64_t* prev = dev_prev ? dev_prev : e->d_prev;
  const int all = full || (!dev_prev && !valid);
  if (wait_stream != TPI_NO_STREAM) {
    HIP_OK(hipEventRecord(e->ev_wait, (hipStream_t)wait_stream));
    HIP_OK(hipStreamWaitEvent(e->compute, e->ev_wait, 0));
  }
  // 1. digests of the current tensors, 2. dirty list (and new digests remembered)
  HIP_OK(tpi_launch_stream_hash(e->d_segs, n, total, tile, TPI_SYNC_SEED, e->d_hash,
                                e->compute));
  HIP_OK(hipMemsetAsync(e->d_count, 0, sizeof(unsigned int), e->compute));
  HIP_OK(tpi_launch_dirty_tiles(e->d_hash, prev, ntiles, all, e->d_idx, e->d_count,
                                e->compute));
  unsigned int count = 0;
  HIP_OK(region_copy(e, &count, e->d_count, sizeof(count), hipMemcpyDeviceToHost, e->compute));
  HIP_OK(hipStreamSynchronize(e->compute));
  std::vector<uint32_t> idx(count);
  if (count) {
    HIP_OK(hipMemcpy(idx.data(), e->d_idx, count * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::sort(idx.begin(), idx.end());  // ascending: consecutive tiles coalesce into one DMA
    HIP_OK(hipMemcpy(e->d_idx, idx.data(), count * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_OK(region_copy(e, e->d_crcs, crcs_inout, ntiles * sizeof(uint32_t),
                          hipMemcpyHostToDevice, e->compute));
  }
  // 3. pack the dirty tiles compactly, 4. DMA each run of consecutive tiles to its place
  const uint32_t init_full = init_for(tile);
  const uint32_t init_last = init_for(total % tile ? total % tile : tile);
  const uint64_t per_buf = e->chunk / tile;
  uint8_t* dst = (uint8_t*)host_dst;
  uint64_t batches = 0;
  for (uint64_t first = 0, k = 0; first < count; first += per_buf, ++k) {
    const int b = (int)(k % e->nbuf);
    const uint32_t m = (uint32_t)std::min<uint64_t>(per_buf, count - first);
    if (k >= (uint64_t)e->nbuf && staging_free(e, b, e->compute)) return -1;
    HIP_OK(tpi_launch_pack_list(e->d_segs, n, total, e->d_idx + first, m, e->staging[b], tile,
                                e->tables, e->d_crcs, init_full, init_last, e->compute));
    if (staging_ready(e, b, e->compute)) return -1;
    for (uint32_t j = 0; j < m;) {
      uint32_t r = j + 1;
      while (r < m && idx[first + r] == idx[first + r - 1] + 1) ++r;
      const uint64_t start = (uint64_t)idx[first + j] * tile;
      const uint64_t end = std::min<uint64_t>(total, (uint64_t)(idx[first + r - 1] + 1) * tile);
      if (staging_d2h(e, b, dst + start, (uint8_t*)e->staging[b] + (uint64_t)j * tile,
                      end - start))
        return -1;
      j = r;
    }
    if (staging_sent(e, b)) return -1;
    batches = k + 1;
  }
  if (count)
    HIP_OK(region_copy(e, crcs_inout, e->d_crcs, ntiles * sizeof(uint32_t),
                          hipMemcpyDeviceToHost, e->compute));
  if (drain_d2h(e)) return -1;
  HIP_OK(hipStreamSynchronize(e->compute));
  if (!dev_prev) {
    e->hash_valid = true;
    e->hash_ntiles = ntiles;
  }
  *dirty_tiles = count;
  if (stats) {
    stats->copy_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats->pack_ms = 0;
    stats->bytes = std::min<uint64_t>(total, (uint64_t)count * tile);
    stats->chunks = batches;
  }
  return 0;
}

}  // extern "C"

namespace {

int prepare_codec(tpi_engine* e, uint64_t ntiles) {
  const uint64_t per_chunk = e->chunk / e->tile;
  if (!e->zraw) {
    HIP_OK(hipMalloc(&e->zraw, e->chunk));
    HIP_OK(hipMalloc(&e->d_meta, tpz_meta_bytes(per_chunk)));
  }
  if (ntiles + 1 > e->z_cap) {
    if (e->d_csize) HIP_OK(hipFree(e->d_csize));
    if (e->d_coff) HIP_OK(hipFree(e->d_coff));
    if (e->h_coff) HIP_OK(hipHostFree(e->h_coff));
    e->d_csize = nullptr;
    e->d_coff = e->h_coff = nullptr;
    e->z_cap = 0;
    const size_t cap = std::max<size_t>(ntiles + 1, 1024);
    HIP_OK(hipMalloc(&e->d_csize, cap * sizeof(uint32_t)));
    HIP_OK(hipMalloc(&e->d_coff, cap * sizeof(uint64_t)));
    HIP_OK(hipHostMalloc(&e->h_coff, cap * sizeof(uint64_t), hipHostMallocDefault));
    e->z_cap = cap;
  }
  return 0;
}

}  // namespace

extern "C" {

// Compressed save: per chunk  pack+CRC -> zraw, analyze+encode -> staging[b] (TPZ1 blobs,
// contiguous), blob sizes -> csizes_out (host);  the host learns the chunk's compressed length
// from those sizes and only then queues its D2H, so PCIe carries the compressed bytes only.
// The host waits on each chunk's (short) compute while the copy stream is still draining the
// previous chunks, so the link stays busy.
int tpi_save_z(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* host_dst,
               uint32_t* crcs_out, uint32_t* csizes_out, uint64_t wait_stream,
               uint64_t* stream_bytes, tpi_stats* stats) {
  Range range("tpi_save_z");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  if (prepare(e, segs, n, total)) return -1;
  const uint64_t tile = e->tile;
  const uint64_t ntiles = (total + tile - 1) / tile;
  if (prepare_codec(e, ntiles)) return -1;
  e->hash_valid = false;
  if (wait_stream != TPI_NO_STREAM) {
    HIP_OK(hipEventRecord(e->ev_wait, (hipStream_t)wait_stream));
    HIP_OK(hipStreamWaitEvent(e->compute, e->ev_wait, 0));
  }
  const uint32_t init_full = init_for(tile);
  const uint32_t init_last = init_for(total % tile ? total % tile : tile);
  uint8_t* dst = (uint8_t*)host_dst;
  uint64_t out = 0, nchunks = 0, published = 0;
  std::vector<ChunkMark> marks;
  // streamed: the kernels store CRCs and blob sizes in the host arrays themselves (meta_view)
  uint32_t* crc_host =
      e->progress ? (uint32_t*)meta_view(e, crcs_out, ntiles * sizeof(uint32_t), false)
                  : nullptr;
  uint32_t* csz_host =
      crc_host ? (uint32_t*)meta_view(e, csizes_out, ntiles * sizeof(uint32_t), false) : nullptr;
  if (!csz_host) crc_host = nullptr;
  for (uint64_t base = 0, k = 0; base < total; base += e->chunk, ++k) {
    const int b = (int)(k % e->nbuf);
    const uint64_t len = std::min(e->chunk, total - base);
    const uint64_t t0i = base / tile, nt = (len + tile - 1) / tile;
    if (k >= (uint64_t)e->nbuf && staging_free(e, b, e->compute)) return -1;
    HIP_OK(tpi_launch_transposes(segs, n, base, len, e->zraw, 0, e->compute));
    HIP_OK(tpi_launch_stream_crc(0, e->d_segs, n, base, len, e->zraw, tile, e->tables,
                                 crc_host ? crc_host : e->d_crcs, init_full, init_last, nullptr,
                                 1, e->compute));
    HIP_OK(tpi_launch_tpz_encode(e->zraw, len, tile, e->d_meta, e->d_csize + t0i,
                                 csz_host ? csz_host + t0i : nullptr, e->staging[b], e->compute));
    if (!csz_host)
      HIP_OK(region_copy(e, csizes_out + t0i, e->d_csize + t0i, nt * sizeof(uint32_t),
                         hipMemcpyDeviceToHost, e->compute));
    HIP_OK(hipEventRecord(e->ev_a[b], e->compute));
    HIP_OK(hipEventSynchronize(e->ev_a[b]));
    uint64_t clen = 0;
    for (uint64_t i = 0; i < nt; ++i) clen += csizes_out[t0i + i];
    if (!e->sdma) HIP_OK(hipStreamWaitEvent(e->copy, e->ev_a[b], 0));
    if (staging_d2h(e, b, dst + out, e->staging[b], clen) || staging_sent(e, b)) return -1;
    out += clen;
    marks.push_back({t0i + nt, out});
    if (e->progress && k >= 1 &&
        publish_chunk(e, marks, k - 1, &published, crc_host ? nullptr : crcs_out))
      return -1;
    nchunks = k + 1;
  }
  if (e->progress && !marks.empty() &&
      publish_chunk(e, marks, marks.size() - 1, &published, crc_host ? nullptr : crcs_out))
    return -1;
  if (!crc_host)
    HIP_OK(region_copy(e, crcs_out, e->d_crcs, ntiles * sizeof(uint32_t), hipMemcpyDeviceToHost,
                       e->compute));
  if (drain_d2h(e)) return -1;
  HIP_OK(hipStreamSynchronize(e->compute));
  *stream_bytes = out;
  if (stats) {
    stats->copy_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats->pack_ms = 0;
    stats->bytes = out;
    stats->chunks = nchunks;
  }
  return 0;
}

// Asynchronous checkpoints, step 1: pack the tensors (+ tile CRCs) into a device snapshot
// buffer, ordered after `wait_stream`'s pending work; `wait_stream` then waits for the pack,
// so training kernels queued afterwards cannot overwrite tensors before they are captured.
// Nothing blocks the host.
int tpi_snapshot(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* dev_dst,
                 uint32_t* dev_crcs, uint64_t wait_stream) {
  Range range("tpi_snapshot");
  std::lock_guard<std::mutex> lk(e->mu);
  if (prepare(e, segs, n, total)) return -1;
  e->hash_valid = false;
  if (wait_stream != TPI_NO_STREAM) {
    HIP_OK(hipEventRecord(e->ev_wait, (hipStream_t)wait_stream));
    HIP_OK(hipStreamWaitEvent(e->compute, e->ev_wait, 0));
  }
  const uint64_t tile = e->tile;
  HIP_OK(tpi_launch_transposes(segs, n, 0, total, dev_dst, 0, e->compute));
  HIP_OK(tpi_launch_stream_crc(0, e->d_segs, n, 0, total, dev_dst, tile, e->tables, dev_crcs,
                               init_for(tile), init_for(total % tile ? total % tile : tile),
                               nullptr, 1, e->compute));
  HIP_OK(hipEventRecord(e->ev_done, e->compute));
  if (wait_stream != TPI_NO_STREAM) HIP_OK(hipStreamWaitEvent((hipStream_t)wait_stream, e->ev_done, 0));
  return 0;
}

// Step 2 (called from a background thread): move a snapshot to host memory, raw or TPZ1
// encoded chunk by chunk, plus its CRCs.  Runs only on the engine's streams, concurrently
// with whatever the training stream does.
int tpi_spill(tpi_engine* e, const void* dev_src, const uint32_t* dev_crcs, uint64_t total,
              void* host_dst, uint32_t* crcs_out, uint32_t* csizes_out, int codec,
              uint64_t* stream_bytes, tpi_stats* stats) {
  Range range("tpi_spill");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  HIP_OK(hipSetDevice(e->device));
  if (e->sdma && tpi_sdma_wait_all(e->sdma)) return -1;
  const uint64_t tile = e->tile;
  const uint64_t ntiles = (total + tile - 1) / tile;
  // the snapshot was packed on `compute`; everything below is ordered after it
  HIP_OK(hipEventRecord(e->ev_wait, e->compute));
  HIP_OK(hipStreamWaitEvent(e->copy, e->ev_wait, 0));
  uint8_t* dst = (uint8_t*)host_dst;
  const uint8_t* src = (const uint8_t*)dev_src;
  uint64_t out = 0, nchunks = 0;
  if (!codec) {
    if (e->sdma) HIP_OK(hipEventSynchronize(e->ev_wait));
    for (uint64_t base = 0; base < total; base += e->chunk, ++nchunks) {
      const uint64_t len = std::min(e->chunk, total - base);
      if (e->sdma) {
        if (sdma_region_d2h(e, e->nbuf, dst + base, src + base, len)) return -1;
      } else {
        HIP_OK(region_copy(e, dst + base, src + base, len, hipMemcpyDeviceToHost, e->copy));
      }
    }
    out = total;
  } else {
    if (prepare_codec(e, ntiles)) return -1;
    for (uint64_t base = 0, k = 0; base < total; base += e->chunk, ++k) {
      const int b = (int)(k % e->nbuf);
      const uint64_t len = std::min(e->chunk, total - base);
      const uint64_t t0i = base / tile, nt = (len + tile - 1) / tile;
      if (k >= (uint64_t)e->nbuf && staging_free(e, b, e->compute)) return -1;
      HIP_OK(tpi_launch_tpz_encode(src + base, len, tile, e->d_meta, e->d_csize + t0i,
                                   nullptr, e->staging[b], e->compute));
      HIP_OK(region_copy(e, csizes_out + t0i, e->d_csize + t0i, nt * sizeof(uint32_t),
                            hipMemcpyDeviceToHost, e->compute));
      HIP_OK(hipEventRecord(e->ev_a[b], e->compute));
      HIP_OK(hipEventSynchronize(e->ev_a[b]));
      uint64_t clen = 0;
      for (uint64_t i = 0; i < nt; ++i) clen += csizes_out[t0i + i];
      if (!e->sdma) HIP_OK(hipStreamWaitEvent(e->copy, e->ev_a[b], 0));
      if (staging_d2h(e, b, dst + out, e->staging[b], clen) || staging_sent(e, b)) return -1;
      out += clen;
      nchunks = k + 1;
    }
  }
  HIP_OK(region_copy(e, crcs_out, dev_crcs, ntiles * sizeof(uint32_t), hipMemcpyDeviceToHost,
                        e->copy));
  if (drain_d2h(e)) return -1;
  HIP_OK(hipStreamSynchronize(e->compute));
  *stream_bytes = out;
  if (stats) {
    stats->copy_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats->pack_ms = 0;
    stats->bytes = out;
    stats->chunks = nchunks;
  }
  return 0;
}

// Compressed restore: H2D of each chunk's blobs -> staging[b], decode -> zraw, unpack+verify.
int tpi_restore_z(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total,
                  const void* host_src, const uint32_t* crcs, const uint32_t* csizes,
                  uint64_t signal_stream, uint64_t* bad_tiles, int64_t* first_bad,
                  tpi_stats* stats) {
  Range range("tpi_restore_z");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  if (prepare(e, segs, n, total)) return -1;
  const uint64_t tile = e->tile;
  const uint64_t ntiles = (total + tile - 1) / tile;
  if (prepare_codec(e, ntiles)) return -1;
  e->hash_valid = false;
  // Blob offsets (pinned); a size that cannot come from the encoder means a corrupt index.
  uint64_t* coff = e->h_coff;
  coff[0] = 0;
  for (uint64_t i = 0; i < ntiles; ++i) {
    const uint64_t tl = std::min(tile, total - i * tile);
    if (csizes[i] < TPZ_HDR || csizes[i] > tpz_bound(tl) || csizes[i] % 16)
      return fail("corrupt compressed index at tile " + std::to_string(i));
    coff[i + 1] = coff[i] + csizes[i];
  }
  const uint32_t init_full = init_for(tile);
  const uint32_t init_last = init_for(total % tile ? total % tile : tile);
  unsigned long long bad_init[2] = {0ull, ~0ull};
  if (signal_stream != TPI_NO_STREAM) {
    HIP_OK(hipEventRecord(e->ev_wait, (hipStream_t)signal_stream));
    HIP_OK(hipStreamWaitEvent(e->compute, e->ev_wait, 0));
  }
  HIP_OK(region_copy(e, e->d_crcs, crcs, ntiles * sizeof(uint32_t), hipMemcpyHostToDevice,
                        e->compute));
  HIP_OK(hipMemcpyAsync(e->d_coff, coff, (ntiles + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                        e->compute));
  HIP_OK(region_copy(e, e->d_bad, bad_init, sizeof(bad_init), hipMemcpyHostToDevice,
                        e->compute));
  HIP_OK(hipEventRecord(e->ev_wait, e->compute));
  HIP_OK(hipStreamWaitEvent(e->copy, e->ev_wait, 0));
  const uint8_t* src = (const uint8_t*)host_src;
  uint64_t nchunks = 0;
  for (uint64_t base = 0, k = 0; base < total; base += e->chunk, ++k) {
    const int b = (int)(k % e->nbuf);
    const uint64_t len = std::min(e->chunk, total - base);
    const uint64_t t0i = base / tile, nt = (len + tile - 1) / tile;
    const uint64_t cbeg = coff[t0i], cend = coff[t0i + nt];
    if (k >= (uint64_t)e->nbuf) HIP_OK(hipStreamWaitEvent(e->copy, e->ev_b[b], 0));
    HIP_OK(region_copy(e, e->staging[b], src + cbeg, cend - cbeg, hipMemcpyHostToDevice,
                          e->copy));
    HIP_OK(hipEventRecord(e->ev_a[b], e->copy));
    HIP_OK(hipStreamWaitEvent(e->compute, e->ev_a[b], 0));
    HIP_OK(tpi_launch_tpz_decode(e->staging[b], e->d_coff + t0i, cbeg, len, tile, e->zraw,
                                 e->compute));
    HIP_OK(hipEventRecord(e->ev_b[b], e->compute));
    HIP_OK(tpi_launch_stream_crc(1, e->d_segs, n, base, len, e->zraw, tile, e->tables,
                                 e->d_crcs, init_full, init_last, e->d_bad, 1, e->compute));
    HIP_OK(tpi_launch_transposes(segs, n, base, len, e->zraw, 1, e->compute));
    nchunks = k + 1;
  }
  unsigned long long bad[2];
  HIP_OK(region_copy(e, bad, e->d_bad, sizeof(bad), hipMemcpyDeviceToHost, e->compute));
  HIP_OK(hipEventRecord(e->ev_done, e->compute));
  if (signal_stream != TPI_NO_STREAM) HIP_OK(hipStreamWaitEvent((hipStream_t)signal_stream, e->ev_done, 0));
  HIP_OK(hipStreamSynchronize(e->compute));
  HIP_OK(hipStreamSynchronize(e->copy));
  HIP_OK(hipStreamSynchronize(e->copy2));
  *bad_tiles = bad[0];
  *first_bad = bad[0] ? (int64_t)bad[1] : -1;
  if (stats) {
    stats->copy_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats->pack_ms = 0;
    stats->bytes = coff[ntiles];
    stats->chunks = nchunks;
  }
  return 0;
}

int tpi_tpz_encode_device(const void* raw, uint64_t len, uint64_t tile, void* meta_scratch,
                          uint32_t* csize, void* out, uint64_t stream) {
  if (tile == 0 || tile % TPI_ROW_BYTES) return fail("tile must be k*4096");
  if (len % 16) return fail("length must be a multiple of 16");
  HIP_OK(tpi_launch_tpz_encode(raw, len, tile, meta_scratch, csize, nullptr, out,
                               (hipStream_t)stream));
  return 0;
}

int tpi_tpz_decode_device(const void* comp, const uint64_t* coff, uint64_t len, uint64_t tile,
                          void* raw, uint64_t stream) {
  if (tile == 0 || tile % TPI_ROW_BYTES) return fail("tile must be k*4096");
  if (len % 16) return fail("length must be a multiple of 16");
  HIP_OK(tpi_launch_tpz_decode(comp, coff, 0, len, tile, raw, (hipStream_t)stream));
  return 0;
}

int tpi_stream_hash(const tpi_seg* dev_segs, int n, uint64_t total, uint64_t tile_bytes,
                    uint64_t seed, uint64_t* dev_out, uint64_t stream) {
  if (tile_bytes == 0 || tile_bytes % TPI_ROW_BYTES) return fail("tile must be k*4096");
  HIP_OK(tpi_launch_stream_hash(dev_segs, n, total, tile_bytes, seed, dev_out,
                                (hipStream_t)stream));
  return 0;
}

int tpi_crc32c_tiles(const void* dev_ptr, uint64_t nbytes, uint64_t tile_bytes,
                     uint32_t* dev_out, uint64_t stream) {
  if (tile_bytes == 0 || tile_bytes % TPI_ROW_BYTES) return fail("tile must be k*4096");
  if (nbytes % 16) return fail("length must be a multiple of 16");
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  tpi_crc_tables* t = nullptr;
  if (device_tables(dev, &t)) return -1;
  const uint32_t init_full = init_for(tile_bytes);
  const uint32_t init_last = init_for(nbytes % tile_bytes ? nbytes % tile_bytes : tile_bytes);
  HIP_OK(tpi_launch_stream_crc(2, nullptr, 0, 0, nbytes, (void*)dev_ptr, tile_bytes, t, dev_out,
                               init_full, init_last, nullptr, 0, (hipStream_t)stream));
  return 0;
}

int tpi_shard_hash(const void* dev_ptr, uint64_t nbytes, uint64_t shard_bytes, uint64_t seed,
                   uint64_t* dev_out, uint64_t stream) {
  if (shard_bytes == 0) return fail("shard_bytes must be positive");
  if ((uintptr_t)dev_ptr % 16 || shard_bytes % 32) return fail("need 16B-aligned data, 32B shards");
  HIP_OK(tpi_launch_shard_hash(dev_ptr, nbytes, shard_bytes, seed, dev_out,
                               (hipStream_t)stream));
  return 0;
}

int tpi_pack_device(const tpi_seg* segs, const tpi_seg* host_segs, int n, uint64_t total,
                    void* dev_dst, uint64_t tile_bytes, uint32_t* dev_crcs, uint64_t stream) {
  // `segs` is a DEVICE array here (the caller owns it); validation happens host-side in the
  // Python wrapper, which builds it.
  if (tile_bytes == 0 || tile_bytes % TPI_ROW_BYTES) return fail("tile must be k*4096");
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  tpi_crc_tables* t = nullptr;
  if (device_tables(dev, &t)) return -1;
  HIP_OK(tpi_launch_transposes(host_segs, n, 0, total, dev_dst, 0, (hipStream_t)stream));
  HIP_OK(tpi_launch_stream_crc(0, segs, n, 0, total, dev_dst, tile_bytes, t, dev_crcs,
                               init_for(tile_bytes),
                               init_for(total % tile_bytes ? total % tile_bytes : tile_bytes),
                               nullptr, host_segs ? 1 : 0, (hipStream_t)stream));
  return 0;
}

int tpi_unpack_device(const tpi_seg* segs, const tpi_seg* host_segs, int n, uint64_t total,
                      void* dev_src, uint64_t tile_bytes, const uint32_t* dev_crcs,
                      uint64_t* dev_bad, uint64_t stream) {
  if (tile_bytes == 0 || tile_bytes % TPI_ROW_BYTES) return fail("tile must be k*4096");
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  tpi_crc_tables* t = nullptr;
  if (device_tables(dev, &t)) return -1;
  HIP_OK(tpi_launch_stream_crc(1, segs, n, 0, total, dev_src, tile_bytes, t,
                               (uint32_t*)dev_crcs, init_for(tile_bytes),
                               init_for(total % tile_bytes ? total % tile_bytes : tile_bytes),
                               (unsigned long long*)dev_bad, host_segs ? 1 : 0,
                               (hipStream_t)stream));
  HIP_OK(tpi_launch_transposes(host_segs, n, 0, total, dev_src, 1, (hipStream_t)stream));
  return 0;
}

// ---- host memory ---------------------------------------------------------------------------

void* tpi_host_map(const char* path, uint64_t bytes, int numa_node, int populate) {
  int fd = -1;
  int flags = MAP_PRIVATE | MAP_ANONYMOUS;
  if (path && *path) {
    fd = open(path, O_RDWR | O_CREAT, 0600);
    if (fd < 0) {
      fail(std::string("open ") + path + ": " + strerror(errno));
      return nullptr;
    }
    struct stat st;
    if (fstat(fd, &st) == 0 && (uint64_t)st.st_size < bytes && ftruncate(fd, bytes) != 0) {
      fail(std::string("ftruncate: ") + strerror(errno));
      close(fd);
      return nullptr;
    }
    flags = MAP_SHARED;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, flags, fd, 0);
  if (fd >= 0) close(fd);
  if (p == MAP_FAILED) {
    fail(std::string("mmap: ") + strerror(errno));
    return nullptr;
  }
  madvise(p, bytes, MADV_HUGEPAGE);
  if (numa_node >= 0 && numa_node < 1024) {
    unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
    mask[numa_node / (8 * sizeof(unsigned long))] |= 1ul << (numa_node % (8 * sizeof(unsigned long)));
    // MPOL_PREFERRED = 1: fall back to other nodes instead of failing under pressure.
    syscall(SYS_mbind, p, bytes, 1, mask, 1024, 0);
  }
  if (populate) {
    // Parallel first touch: page faults dominate, one thread per ~1 GiB up to 16.
    const uint64_t page = 4096;
    unsigned nth = (unsigned)std::min<uint64_t>(16, std::max<uint64_t>(1, bytes >> 30));
    std::vector<std::thread> th;
    const uint64_t per = ((bytes / nth) + page - 1) / page * page;
    for (unsigned i = 0; i < nth; ++i) {
      th.emplace_back([=] {
        uint64_t b = (uint64_t)i * per, e = std::min(bytes, b + per);
        volatile uint8_t* q = (volatile uint8_t*)p;
        for (uint64_t o = b; o < e; o += page) q[o] = q[o];
      });
    }
    for (auto& t : th) t.join();
  }
  return p;
}

int tpi_host_unmap(void* ptr, uint64_t bytes) {
  if (munmap(ptr, bytes)) return fail(std::string("munmap: ") + strerror(errno));
  return 0;
}

int tpi_host_register(void* ptr, uint64_t bytes) {
  HIP_OK(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  return 0;
}

int tpi_host_register_ro(void* ptr, uint64_t bytes) {
  HIP_OK(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterReadOnly));
  return 0;
}

int tpi_h2d_async(void* dev_dst, const void* host_src, uint64_t bytes, uint64_t stream) {
  HIP_OK(hipMemcpyAsync(dev_dst, host_src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return 0;
}

tpi_pinner* tpi_host_pin_start(void* base, uint64_t bytes, uint64_t window, int threads) {
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) device = 0;
  auto* p = new tpi_pinner();
  p->base = (uint8_t*)base;
  p->bytes = bytes;
  p->window = std::max<uint64_t>(2ull << 20, window / (2ull << 20) * (2ull << 20));
  p->threads = std::max(1, threads);
  p->device = device;
  p->toucher = std::thread([p] {
    constexpr uint64_t page = 4096;
    for (uint64_t w = 0; w < p->bytes && !p->stop.load(); w += p->window) {
      const uint64_t end = std::min(p->bytes, w + p->window);
      const uint64_t per = ((end - w) / p->threads + page - 1) / page * page;
      std::vector<std::thread> pool;
      for (int t = 0; t < p->threads; ++t)
        pool.emplace_back([p, w, end, per, t] {
          const uint64_t b = w + (uint64_t)t * per, e = std::min(end, b + per);
          volatile const uint8_t* q = p->base;
          uint8_t sink = 0;
          for (uint64_t o = b; o < e; o += page) sink ^= q[o];  // read fault: no data change
          (void)sink;
        });
      for (auto& t : pool) t.join();
      p->touched.store(end, std::memory_order_release);
    }
  });
  p->registrar = std::thread([p] {
    (void)hipSetDevice(p->device);
    for (uint64_t w = 0; w < p->bytes && !p->stop.load(); w += p->window) {
      const uint64_t end = std::min(p->bytes, w + p->window);
      while ((p->touched.load(std::memory_order_acquire) < end ||
              p->held.load(std::memory_order_acquire)) && !p->stop.load())
        std::this_thread::sleep_for(std::chrono::microseconds(100));
      if (p->stop.load()) break;
      hipError_t err = hipHostRegister(p->base + w, end - w,
                                       hipHostRegisterMapped | hipHostRegisterPortable);
      if (err != hipSuccess) {
        p->error = std::string("hipHostRegister(window) : ") + hipGetErrorString(err);
        p->failed.store(true);
        return;
      }
      p->registered.push_back(p->base + w);
      p->ready.store(end, std::memory_order_release);
    }
  });
  return p;
}

uint64_t tpi_host_pin_ready(const tpi_pinner* p) { return p->ready.load(); }

int tpi_host_pin_hold(tpi_pinner* p, int hold) {
  p->held.store(hold != 0, std::memory_order_release);
  return 0;
}
uint64_t tpi_host_pin_window(const tpi_pinner* p) { return p->window; }

// Wait for the whole region (0) or report the pinning error (-1).
int tpi_host_pin_wait(tpi_pinner* p) {
  p->held.store(false, std::memory_order_release);
  if (p->toucher.joinable()) p->toucher.join();
  if (p->registrar.joinable()) p->registrar.join();
  if (p->failed.load()) return fail(p->error);
  return 0;
}

// Stop (if still running), unregister every pinned window, free the pinner.
int tpi_host_pin_release(tpi_pinner* p) {
  if (!p) return 0;
  p->stop.store(true);
  if (p->toucher.joinable()) p->toucher.join();
  if (p->registrar.joinable()) p->registrar.join();
  for (uint8_t* w : p->registered) (void)hipHostUnregister(w);
  delete p;
  return 0;
}

int tpi_engine_set_host_region(tpi_engine* e, void* base, uint64_t bytes, uint64_t window,
                               tpi_pinner* pinner) {
  std::lock_guard<std::mutex> lk(e->mu);
  e->hbase = (const uint8_t*)base;
  e->hbytes = bytes;
  e->hwin = window;
  e->pinner = pinner;
  return 0;
}

// Allocate now what the pipelines would allocate on first use (segment descriptors, tile
// CRCs, the codec's decode buffers): a successor that restores while its predecessor frees
// HBM must not meet a hipMalloc that waits for the driver to clear that memory.
int tpi_engine_reserve(tpi_engine* e, int nsegs, uint64_t ntiles, int codec) {
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_OK(hipSetDevice(e->device));
  if ((size_t)nsegs > e->seg_cap) {
    if (e->d_segs) HIP_OK(hipFree(e->d_segs));
    e->d_segs = nullptr;
    e->seg_cap = 0;
    HIP_OK(hipMalloc(&e->d_segs, (size_t)nsegs * sizeof(tpi_seg)));
    e->seg_cap = nsegs;
  }
  if (ntiles > e->crc_cap) {
    if (e->d_crcs) HIP_OK(hipFree(e->d_crcs));
    e->d_crcs = nullptr;
    e->crc_cap = 0;
    HIP_OK(hipMalloc(&e->d_crcs, ntiles * sizeof(uint32_t)));
    e->crc_cap = ntiles;
  }
  // the HBM hand-off's buffers as well: a successor's first copy then allocates nothing
  if (ntiles > e->digest_cap) {
    if (e->d_digest) HIP_OK(hipFree(e->d_digest));
    e->d_digest = nullptr;
    e->digest_cap = 0;
    HIP_OK(hipMalloc(&e->d_digest, ntiles * sizeof(uint64_t)));
    e->digest_cap = ntiles;
  }
  if ((size_t)nsegs > e->src_cap) {
    if (e->d_src) HIP_OK(hipFree(e->d_src));
    e->d_src = nullptr;
    e->src_cap = 0;
    HIP_OK(hipMalloc(&e->d_src, (size_t)nsegs * sizeof(tpi_seg)));
    e->src_cap = nsegs;
  }
  if (codec && prepare_codec(e, ntiles)) return -1;
  return 0;
}

int tpi_engine_set_h2d_sdma(tpi_engine* e, int on) {
  std::lock_guard<std::mutex> lk(e->mu);
  if (!on) {
    tpi_sdma_close(e->sdma_in);
    e->sdma_in = nullptr;
    return 0;
  }
  if (!e->sdma_in) e->sdma_in = tpi_sdma_open_h2d(e->device, e->nbuf);
  return e->sdma_in ? (int)(31 - __builtin_clz(tpi_sdma_engine(e->sdma_in))) : -1;
}

int tpi_engine_set_progress(tpi_engine* e, uint64_t* words) {
  std::lock_guard<std::mutex> lk(e->mu);
  e->progress = words;
  return 0;
}

// Restore from a region another process is still writing (streaming hand-off): the same
// pipeline as tpi_restore / tpi_restore_z, but chunk k's H2D starts only once the writer has
// published its tiles (progress words[0]); its CRCs (and blob sizes) are read from the host
// then, and uploaded per chunk.  csizes == NULL: raw stream.
int tpi_restore_stream(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total,
                       const void* host_src, const uint32_t* crcs, const uint32_t* csizes,
                       const uint64_t* words, double timeout_s, uint64_t signal_stream,
                       uint64_t* bad_tiles, int64_t* first_bad, tpi_stats* stats) {
  return tpi_restore_stream_at(e, segs, n, total, host_src, crcs, csizes, words, 0, timeout_s,
                               signal_stream, bad_tiles, first_bad, stats);
}

// The same for a stretch of the writer's stream starting at its tile `tile_base` (a
// progressive restore allocates and restores the state group by group: the plan, `host_src`,
// `crcs` and `csizes` describe the stretch, the progress words count the whole stream's tiles).
int tpi_restore_stream_at(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total,
                          const void* host_src, const uint32_t* crcs, const uint32_t* csizes,
                          const uint64_t* words, uint64_t tile_base, double timeout_s,
                          uint64_t signal_stream, uint64_t* bad_tiles, int64_t* first_bad,
                          tpi_stats* stats) {
  Range range("tpi_restore_stream");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  if (prepare(e, segs, n, total)) return -1;
  const uint64_t tile = e->tile;
  const uint64_t ntiles = (total + tile - 1) / tile;
  const bool zipped = csizes != nullptr;
  if (zipped && prepare_codec(e, ntiles)) return -1;
  e->hash_valid = false;
  const uint32_t init_full = init_for(tile);
  const uint32_t init_last = init_for(total % tile ? total % tile : tile);
  unsigned long long bad_init[2] = {0ull, ~0ull};
  if (signal_stream != TPI_NO_STREAM) {
    HIP_OK(hipEventRecord(e->ev_wait, (hipStream_t)signal_stream));
    HIP_OK(hipStreamWaitEvent(e->compute, e->ev_wait, 0));
  }
  HIP_OK(region_copy(e, e->d_bad, bad_init, sizeof(bad_init), hipMemcpyHostToDevice,
                     e->compute));
  // blob offsets: pinned, so each chunk's slice goes up asynchronously (a pageable source
  // made every per-chunk copy wait for the copy stream to drain: ~1 ms of idle link a chunk)
  uint64_t* coff = zipped ? e->h_coff : nullptr;
  std::vector<uint64_t> raw_coff;
  if (!zipped) {
    raw_coff.assign(ntiles + 1, 0);
    coff = raw_coff.data();
  }
  coff[0] = 0;
  // the kernels read the writer's CRCs and the blob offsets where they are (meta_view), so no
  // per-chunk uploads on the aux stream
  const uint32_t* crc_host =
      (const uint32_t*)meta_view(e, crcs, ntiles * sizeof(uint32_t), true);
  const uint64_t* coff_host =
      zipped && crc_host
          ? (const uint64_t*)meta_view(e, e->h_coff, (ntiles + 1) * sizeof(uint64_t), true)
          : nullptr;
  const bool direct = crc_host && (!zipped || coff_host);
  uint32_t* crc_src = direct ? (uint32_t*)crc_host : e->d_crcs;
  const uint8_t* src = (const uint8_t*)host_src;
  uint64_t nchunks = 0;
  const uint64_t chunk_tiles = e->chunk / tile;
  std::vector<bool> was_split(e->nbuf, false);
  e->split_chunks = 0;
  // H2D on the engine's own SDMA lanes (tpi_engine_set_h2d_sdma): the host issues chunk k's
  // copy, then waits for chunk k-1's and queues its kernels (a HIP stream cannot wait on the
  // lane's signal); needs two staging buffers at least
  const bool sdma_in = e->sdma_in != nullptr && e->nbuf >= 2;
  struct Pending {
    bool valid;
    int b;
    uint64_t base, len, t0i, cbeg;
  } pending{false, 0, 0, 0, 0, 0};
  auto kernels = [&](const Pending& c) -> int {
    if (!direct) HIP_OK(hipStreamWaitEvent(e->compute, e->ev_c[c.b], 0));
    if (zipped) {
      HIP_OK(tpi_launch_tpz_decode(e->staging[c.b], (direct ? coff_host : e->d_coff) + c.t0i,
                                   c.cbeg, c.len, tile, e->zraw, e->compute));
      HIP_OK(hipEventRecord(e->ev_b[c.b], e->compute));
      HIP_OK(tpi_launch_stream_crc(1, e->d_segs, n, c.base, c.len, e->zraw, tile, e->tables,
                                   crc_src, init_full, init_last, e->d_bad, 1, e->compute));
      HIP_OK(tpi_launch_transposes(segs, n, c.base, c.len, e->zraw, 1, e->compute));
    } else {
      HIP_OK(tpi_launch_stream_crc(1, e->d_segs, n, c.base, c.len, e->staging[c.b], tile,
                                   e->tables, crc_src, init_full, init_last, e->d_bad, 1,
                                   e->compute));
      HIP_OK(tpi_launch_transposes(segs, n, c.base, c.len, e->staging[c.b], 1, e->compute));
      HIP_OK(hipEventRecord(e->ev_b[c.b], e->compute));
    }
    return 0;
  };
  for (uint64_t base = 0, k = 0; base < total; base += e->chunk, ++k) {
    const int b = (int)(k % e->nbuf);
    const uint64_t len = std::min(e->chunk, total - base);
    const uint64_t t0i = base / tile, nt = (len + tile - 1) / tile;
    if (wait_published(words, tile_base + t0i + nt, timeout_s)) {
      // leave no copy or kernel of the chunks already issued running past this call
      (void)hipStreamSynchronize(e->copy);
      (void)hipStreamSynchronize(e->copy2);
      (void)hipStreamSynchronize(e->aux);
      (void)hipStreamSynchronize(e->compute);
      if (sdma_in) (void)tpi_sdma_wait_all(e->sdma_in);
      return -1;
    }
    // How far the restore trails the writer.  The host may run at most nbuf chunks ahead of
    // the copies (wait for chunk k - nbuf's H2D), so the chunks published past this one are
    // the copies' real backlog.  A backlog of split_lead chunks means the save is taking the
    // larger share of the link: split this chunk's H2D over two streams (two SDMA engines).
    if (k >= (uint64_t)e->nbuf && !sdma_in) {
      HIP_OK(hipEventSynchronize(e->ev_a[b]));
      if (was_split[b]) HIP_OK(hipEventSynchronize(e->ev_d[b]));
    }
    const uint64_t published = __atomic_load_n(&words[0], __ATOMIC_ACQUIRE) - tile_base;
    const bool split = chunk_tiles > 0 && published >= t0i + nt &&
                       (published - (t0i + nt)) / chunk_tiles >= e->split_lead;
    uint64_t cbeg = base, cend = base + len;
    if (zipped) {
      for (uint64_t i = t0i; i < t0i + nt; ++i) {
        const uint64_t tl = std::min(tile, total - i * tile);
        if (csizes[i] < TPZ_HDR || csizes[i] > tpz_bound(tl) || csizes[i] % 16)
          return fail("corrupt compressed index at tile " + std::to_string(i));
        coff[i + 1] = coff[i] + csizes[i];
      }
      cbeg = coff[t0i];
      cend = coff[t0i + nt];
    }
    // The chunk's CRCs (and blob offsets) go up on their own stream (see tpi_engine::aux),
    // which the kernels that read them wait for.  On the copy or compute stream these small
    // copies held this thread until the previous chunk's H2D / kernels were done, leaving the
    // link idle ~1 ms per chunk (rocprofv3 memory-copy trace of bench.py).  Slices of
    // different chunks are disjoint (the shared boundary offset is rewritten with the same
    // value).
    if (!direct) {
      if (zipped)
        HIP_OK(hipMemcpyAsync(e->d_coff + t0i, coff + t0i, (nt + 1) * sizeof(uint64_t),
                              hipMemcpyHostToDevice, e->aux));
      HIP_OK(region_copy(e, e->d_crcs + t0i, crcs + t0i, nt * sizeof(uint32_t),
                         hipMemcpyHostToDevice, e->aux));
      HIP_OK(hipEventRecord(e->ev_c[b], e->aux));
    }
    if (sdma_in) {
      // staging[b] is free once chunk k - nbuf's kernels have read it
      if (k >= (uint64_t)e->nbuf) HIP_OK(hipEventSynchronize(e->ev_b[b]));
      if (sdma_region_h2d(e, b, e->staging[b], src + cbeg, cend - cbeg)) {
        (void)tpi_sdma_wait_all(e->sdma_in);
        return -1;
      }
      if (pending.valid) {
        if (tpi_sdma_wait(e->sdma_in, pending.b) || kernels(pending)) {
          (void)tpi_sdma_wait_all(e->sdma_in);
          return -1;
        }
      }
      pending = Pending{true, b, base, len, t0i, cbeg};
      nchunks = k + 1;
      continue;
    }
    if (k >= (uint64_t)e->nbuf) HIP_OK(hipStreamWaitEvent(e->copy, e->ev_b[b], 0));
    // halves split on a 64 KiB boundary of the wire stream (chunks under 128 KiB stay whole)
    const uint64_t mid = split && cend - cbeg >= (128ull << 10)
                             ? cbeg + ((cend - cbeg) / 2 & ~0xFFFFull) : cend;
    HIP_OK(region_copy(e, e->staging[b], src + cbeg, mid - cbeg, hipMemcpyHostToDevice,
                       e->copy));
    HIP_OK(hipEventRecord(e->ev_a[b], e->copy));
    was_split[b] = mid < cend;
    if (was_split[b]) {
      if (k >= (uint64_t)e->nbuf) HIP_OK(hipStreamWaitEvent(e->copy2, e->ev_b[b], 0));
      HIP_OK(region_copy(e, (uint8_t*)e->staging[b] + (mid - cbeg), src + mid, cend - mid,
                         hipMemcpyHostToDevice, e->copy2));
      HIP_OK(hipEventRecord(e->ev_d[b], e->copy2));
      HIP_OK(hipStreamWaitEvent(e->compute, e->ev_d[b], 0));
      ++e->split_chunks;
    }
    HIP_OK(hipStreamWaitEvent(e->compute, e->ev_a[b], 0));
    if (kernels(Pending{true, b, base, len, t0i, cbeg})) return -1;
    nchunks = k + 1;
  }
  if (sdma_in && pending.valid) {
    if (tpi_sdma_wait(e->sdma_in, pending.b) || kernels(pending)) {
      (void)tpi_sdma_wait_all(e->sdma_in);
      return -1;
    }
  }
  unsigned long long bad[2];
  HIP_OK(region_copy(e, bad, e->d_bad, sizeof(bad), hipMemcpyDeviceToHost, e->compute));
  HIP_OK(hipEventRecord(e->ev_done, e->compute));
  if (signal_stream != TPI_NO_STREAM)
    HIP_OK(hipStreamWaitEvent((hipStream_t)signal_stream, e->ev_done, 0));
  HIP_OK(hipStreamSynchronize(e->compute));
  HIP_OK(hipStreamSynchronize(e->copy));
  HIP_OK(hipStreamSynchronize(e->copy2));
  *bad_tiles = bad[0];
  *first_bad = bad[0] ? (int64_t)bad[1] : -1;
  if (stats) {
    stats->copy_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats->pack_ms = 0;
    stats->bytes = zipped ? coff[ntiles] : total;
    stats->chunks = nchunks;
  }
  return 0;
}

// ---- HBM-to-HBM hand-off (preemption on the same GPU) --------------------------------------
// The preempted rank exports its tensors' allocations with HIP IPC; its successor -- a new
// process on the same GPU -- opens them and moves the state device to device through the
// pack / unpack kernels (CRC-verified), instead of waiting for the host spill.

int tpi_mem_range(const void* ptr, uint64_t* base_out, uint64_t* alloc_bytes_out) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  HIP_OK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr));
  *base_out = (uint64_t)(uintptr_t)base;
  *alloc_bytes_out = size;
  return 0;
}

int tpi_ipc_export(const void* ptr, void* handle_out, uint64_t* offset_out,
                   uint64_t* alloc_bytes_out) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  HIP_OK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr));
  hipIpcMemHandle_t h;
  HIP_OK(hipIpcGetMemHandle(&h, (void*)base));
  memcpy(handle_out, &h, sizeof(h));
  *offset_out = (uint64_t)((const uint8_t*)ptr - (const uint8_t*)base);
  *alloc_bytes_out = size;
  return 0;
}

// Move tensors `src` -> `dst` (same plan, different pointers) on the device.  Default: per
// chunk, one fused pass copies tensor to tensor and records the tile CRCs of what it read
// (MODE_COPY), then a read-back pass checks dst against them (MODE_VERIFY): 3 x the state in
// HBM traffic.
// TPI_HANDOFF_COPY=staged (or segments whose stream layouts differ) takes the older route:
// pack src into a staging buffer, then unpack + verify into dst (4 x the traffic).
int tpi_copy_segments(tpi_engine* e, const tpi_seg* src, const tpi_seg* dst, int n,
                      uint64_t total, uint64_t signal_stream, uint64_t* bad_tiles,
                      tpi_stats* stats) {
  Range range("tpi_copy_segments");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  if (check_segments(src, n, total)) return -1;
  if (prepare(e, dst, n, total)) return -1;  // dst -> d_segs
  hipStream_t cs = e->compute;  // the stream of this copy (TPI_HANDOFF_PRIORITY)
  if (e->urgent) {  // after the descriptor upload prepare() queued on `compute`
    HIP_OK(hipEventRecord(e->ev_prio, e->compute));
    HIP_OK(hipStreamWaitEvent(e->urgent, e->ev_prio, 0));
    cs = e->urgent;
  }
  e->hash_valid = false;
  if ((size_t)n > e->src_cap) {  // grown, never shrunk: no allocation per hand-off
    if (e->d_src) HIP_OK(hipFree(e->d_src));
    e->d_src = nullptr;
    e->src_cap = 0;
    HIP_OK(hipMalloc(&e->d_src, std::max<size_t>(n, 64) * sizeof(tpi_seg)));
    e->src_cap = std::max<size_t>(n, 64);
  }
  tpi_seg* d_src = e->d_src;
  auto release = [&] {};
  auto ok = [&](hipError_t err, const char* what) {
    if (err == hipSuccess) return true;
    fail(std::string(what) + ": " + hipGetErrorString(err));
    return false;
  };
  const uint64_t tile = e->tile;
  const uint32_t init_full = init_for(tile);
  const uint32_t init_last = init_for(total % tile ? total % tile : tile);
  unsigned long long bad_init[2] = {0ull, ~0ull}, bad[2] = {0ull, 0ull};
  bool good = ok(hipMemcpyAsync(d_src, src, (size_t)n * sizeof(tpi_seg), hipMemcpyHostToDevice,
                                cs), "upload source segments") &&
              ok(hipMemcpyAsync(e->d_bad, bad_init, sizeof(bad_init), hipMemcpyHostToDevice,
                                cs), "upload bad counter");
  if (good && signal_stream != TPI_NO_STREAM) {  // dst tensors: after the caller's work on them
    good = ok(hipEventRecord(e->ev_wait, (hipStream_t)signal_stream), "hipEventRecord") &&
           ok(hipStreamWaitEvent(cs, e->ev_wait, 0), "hipStreamWaitEvent");
  }
  // device time of the kernels alone (stats->pack_ms): what the hand-off spends beside them
  // (descriptor uploads, host checks, synchronisation) is copy_ms - pack_ms
  if (good) good = ok(hipEventRecord(e->ev_t0, cs), "hipEventRecord");
  bool fused = true;
  for (int i = 0; i < n && fused; ++i)
    fused = src[i].off == dst[i].off && src[i].nbytes == dst[i].nbytes;
  if (const char* m = getenv("TPI_HANDOFF_COPY")) fused = fused && strcmp(m, "staged") != 0;
  // The fused route's tile digest: the XXH64-class stream hash (no table lookups, reads at
  // ~6 TB/s) by default; TPI_HANDOFF_HASH=crc32c keeps the CRC32C tile kernels (~4.3 TB/s
  // read-back, LDS-lookup bound).
  const char* hash_env = getenv("TPI_HANDOFF_HASH");
  const bool xxh = !(hash_env && strcmp(hash_env, "crc32c") == 0);
  const uint64_t ntiles = (total + tile - 1) / tile;
  if (good && fused && xxh && ntiles > e->digest_cap) {
    if (e->d_digest) good = ok(hipFree(e->d_digest), "hipFree(digests)");
    e->d_digest = nullptr;
    e->digest_cap = 0;
    good = good && ok(hipMalloc(&e->d_digest, std::max<uint64_t>(ntiles, 1024) * sizeof(uint64_t)),
                      "hipMalloc(digests)");
    if (good) e->digest_cap = std::max<uint64_t>(ntiles, 1024);
  }
  // How the destination is verified (TPI_HANDOFF_VERIFY): "readback" -- a second pass
  // re-hashes the destination and compares digests; "inline" -- the copy kernel reads every
  // stored word back one row group later and compares it (no second pass over HBM; needs
  // disjoint destinations, else readback); "none" -- unverified (measurement only).
  // profiles/round5/handoff_kernels.md
  const char* verify_env = getenv("TPI_HANDOFF_VERIFY");
  std::string verify = verify_env ? verify_env : "readback";
  if (verify == "inline" && !extents_disjoint(dst, n)) verify = "readback";
  const bool readback = verify == "readback";
  const bool inline_check = verify == "inline";
  uint64_t nchunks = 0;
  // No staging buffer bounds the fused route's spans (a 256 MB chunk would be one workgroup
  // per CU).
  // TPI_HANDOFF_SPAN_MB: bytes per launch; default (0) the whole state in one copy launch and
  // one verify launch -- no launch tails between spans (32 GB: 16.6 ms vs 17.9 ms in 4 GiB
  // spans, profiles/round5/handoff_kernels.md)
  uint64_t span_bytes = total;
  if (const char* v = getenv("TPI_HANDOFF_SPAN_MB"))
    span_bytes = strtoull(v, nullptr, 10) ? strtoull(v, nullptr, 10) << 20 : total;
  // whole tiles, rounded up: the default covers the state's last partial tile in the same
  // launch (rounded down, a second pair of 1-tile launches followed every copy)
  const uint64_t span =
      std::max<uint64_t>(e->chunk, std::max<uint64_t>((span_bytes + tile - 1) / tile, 1) * tile);
  for (uint64_t base = 0, k = 0; good && fused && base < total; base += span, ++k) {
    const uint64_t len = std::min(span, total - base);
    if (xxh)
      good = ok(tpi_launch_stream_copy_hash(d_src, e->d_segs, n, base, len, total, tile,
                                            TPI_SYNC_SEED, e->d_digest,
                                            inline_check ? e->d_bad : nullptr, cs),
                "copy") &&
             (!readback ||
              ok(tpi_launch_stream_copy_hash(e->d_segs, nullptr, n, base, len, total, tile,
                                             TPI_SYNC_SEED, e->d_digest, e->d_bad, cs),
                 "verify"));
    else
      good = ok(tpi_launch_stream_copy(d_src, e->d_segs, n, base, len, tile, e->tables,
                                       e->d_crcs, init_full, init_last, nullptr, cs),
                "copy") &&
             ok(tpi_launch_stream_copy(e->d_segs, nullptr, n, base, len, tile, e->tables,
                                       e->d_crcs, init_full, init_last, e->d_bad, cs),
                "verify");
    nchunks = k + 1;
  }
  for (uint64_t base = 0, k = 0; good && !fused && base < total; base += e->chunk, ++k) {
    const uint64_t len = std::min(e->chunk, total - base);
    void* buf = e->staging[k % e->nbuf];
    good = ok(tpi_launch_transposes(src, n, base, len, buf, 0, cs), "transpose in") &&
           ok(tpi_launch_stream_crc(0, d_src, n, base, len, buf, tile, e->tables, e->d_crcs,
                                    init_full, init_last, nullptr, 1, cs), "pack") &&
           ok(tpi_launch_stream_crc(1, e->d_segs, n, base, len, buf, tile, e->tables,
                                    e->d_crcs, init_full, init_last, e->d_bad, 1, cs),
              "unpack") &&
           ok(tpi_launch_transposes(dst, n, base, len, buf, 1, cs), "transpose out");
    nchunks = k + 1;
  }
  if (good) good = ok(hipEventRecord(e->ev_t1, cs), "hipEventRecord");
  if (good)
    good = ok(hipMemcpyAsync(bad, e->d_bad, sizeof(bad), hipMemcpyDeviceToHost, cs),
              "bad counter") &&
           ok(hipEventRecord(e->ev_done, cs), "hipEventRecord");
  if (good && signal_stream != TPI_NO_STREAM)
    good = ok(hipStreamWaitEvent((hipStream_t)signal_stream, e->ev_done, 0), "hipStreamWaitEvent");
  if (!ok(hipStreamSynchronize(cs), "hipStreamSynchronize")) good = false;
  release();
  if (!good) return -1;
  *bad_tiles = bad[0];
  if (stats) {
    stats->copy_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    float kernel_ms = 0.f;
    stats->pack_ms = hipEventElapsedTime(&kernel_ms, e->ev_t0, e->ev_t1) == hipSuccess ? kernel_ms : -1.0;
    stats->bytes = total;
    stats->chunks = nchunks;
  }
  return 0;
}

int tpi_host_unregister(void* ptr) {
  HIP_OK(hipHostUnregister(ptr));
  return 0;
}

int tpi_h2d(tpi_engine* e, void* dev_dst, const void* host_src, uint64_t bytes) {
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(region_copy(e, dev_dst, host_src, bytes, hipMemcpyHostToDevice, e->copy));
  HIP_OK(hipStreamSynchronize(e->copy));
  return 0;
}

int tpi_d2h(tpi_engine* e, void* host_dst, const void* dev_src, uint64_t bytes) {
  std::lock_guard<std::mutex> lk(e->mu);
  HIP_OK(hipSetDevice(e->device));
  if (e->sdma) {
    if (sdma_region_d2h(e, e->nbuf, host_dst, dev_src, bytes)) return -1;
    return tpi_sdma_wait(e->sdma, e->nbuf);
  }
  HIP_OK(region_copy(e, host_dst, dev_src, bytes, hipMemcpyDeviceToHost, e->copy));
  HIP_OK(hipStreamSynchronize(e->copy));
  return 0;
}

}  // extern "C"
