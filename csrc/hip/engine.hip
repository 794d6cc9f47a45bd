// Host side of libtpi_hip.so, part 1 of the engine: the per-device engine (streams,
// staging ring, CRC tables), device queries, and the helpers its pipelines share
// (engine_internal.h).  The pipelines: engine_save.hip (tpi_save, tpi_sync, tpi_save_z,
// tpi_snapshot, tpi_spill), engine_restore.hip (tpi_restore, tpi_restore_z,
// tpi_restore_stream[_at]), engine_host.hip (pinned host regions), engine_handoff.hip (the
// HBM-to-HBM hand-off copy and the device-side codec / hash entry points).
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
#include "engine_internal.h"

namespace {
thread_local std::string g_err;
}  // namespace

// Error reporting for every translation unit of the library (internal.h).
int tpi_fail(const std::string& what) {
  g_err = what;
  return -1;
}

namespace tpi_engine_detail {



const tpi_crc_tables& host_tables() {
  static tpi_crc_tables t;
  static std::once_flag once;
  std::call_once(once, [] { tpi_crc_tables_init(&t); });
  return t;
}

// Device copies of the CRC tables, one per device (lazily created, never freed).  The
// bank-column layout (TPI_CRC_COLS_WORDS dwords, tpi_crc_cols_init) follows the struct in
// the same allocation: the CRC-only kernel reads it at `tables + 1`.
namespace {
std::mutex g_tab_mu;
std::vector<tpi_crc_tables*> g_dev_tables;
}  // namespace

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


int ensure_staging(tpi_engine* e) {
  for (auto& buf : e->staging)
    if (!buf) HIP_OK(hipMalloc(&buf, e->staging_bytes));
  return 0;
}

int prepare(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, bool staging) {
  if (check_segments(segs, n, total)) return -1;
  HIP_OK(hipSetDevice(e->device));
  if (staging && ensure_staging(e)) return -1;
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

}  // namespace tpi_engine_detail

using namespace tpi_engine_detail;

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
  e->staging.assign(nbuf, nullptr);  // allocated by the first pipeline (ensure_staging)
  e->staging_bytes = staging_bytes;
  e->ev_a.assign(nbuf, nullptr);
  e->ev_b.assign(nbuf, nullptr);
  e->ev_c.assign(nbuf, nullptr);
  e->ev_d.assign(nbuf, nullptr);
  for (int i = 0; i < nbuf; ++i) {
    if ((err = hipEventCreateWithFlags(&e->ev_c[i], hipEventDisableTiming)) != hipSuccess)
      return bail("hipEventCreate", err);
    if ((err = hipEventCreateWithFlags(&e->ev_d[i], hipEventDisableTiming)) != hipSuccess)
      return bail("hipEventCreate", err);
    if ((err = hipEventCreateWithFlags(&e->ev_a[i], hipEventDisableTiming)) != hipSuccess)
      return bail("hipEventCreate", err);
    if ((err = hipEventCreateWithFlags(&e->ev_b[i], hipEventDisableTiming)) != hipSuccess)
      return bail("hipEventCreate", err);
  }
  step("events");
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
