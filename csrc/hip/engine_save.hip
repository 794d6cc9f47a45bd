// Save pipelines of the engine (engine_internal.h): tpi_save (SDMA-staged or direct), tpi_sync
// (incremental: only tiles whose device digest changed cross PCIe), tpi_save_z (TPZ1 codec:
// PCIe carries the compressed bytes only), tpi_snapshot + tpi_spill (asynchronous saves).
// Staged: chunk k packs (+ tile CRCs) into staging[k % nbuf] while chunk k-1 crosses PCIe.
#include "engine_internal.h"

using namespace tpi_engine_detail;

extern "C" {

int tpi_save(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* host_dst,
             uint32_t* crcs_out, int mode, uint64_t wait_stream, tpi_stats* stats) {
  TpiRange range("tpi_save");
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

int tpi_sync(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* host_dst,
             uint32_t* crcs_inout, uint64_t* dev_prev, int full, uint64_t wait_stream,
             uint64_t* dirty_tiles, tpi_stats* stats) {
  TpiRange range("tpi_sync");
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

// Compressed save: per chunk  pack+CRC -> zraw, analyze+encode -> staging[b] (TPZ1 blobs,
// contiguous), blob sizes -> csizes_out (host);  the host learns the chunk's compressed length
// from those sizes and only then queues its D2H, so PCIe carries the compressed bytes only.
// The host waits on each chunk's (short) compute while the copy stream is still draining the
// previous chunks, so the link stays busy.
int tpi_save_z(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* host_dst,
               uint32_t* crcs_out, uint32_t* csizes_out, uint64_t wait_stream,
               uint64_t* stream_bytes, tpi_stats* stats) {
  TpiRange range("tpi_save_z");
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
  TpiRange range("tpi_snapshot");
  std::lock_guard<std::mutex> lk(e->mu);
  if (prepare(e, segs, n, total, false)) return -1;
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
  TpiRange range("tpi_spill");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  HIP_OK(hipSetDevice(e->device));
  if (e->sdma && tpi_sdma_wait_all(e->sdma)) return -1;
  if (ensure_staging(e)) return -1;
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

}  // extern "C"
