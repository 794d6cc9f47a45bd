// Restore pipelines of the engine (engine_internal.h): tpi_restore, tpi_restore_z (TPZ1),
// and tpi_restore_stream[_at] -- a restore behind a save another process is still
// publishing (the streamed preemption hand-off).  H2D on the copy stream(s), unpack + CRC
// verify on the compute stream.
#include "engine_internal.h"

using namespace tpi_engine_detail;

extern "C" {

int tpi_restore(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, const void* host_src,
                const uint32_t* crcs, int mode, uint64_t signal_stream, uint64_t* bad_tiles,
                int64_t* first_bad, tpi_stats* stats) {
  TpiRange range("tpi_restore");
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

// Compressed restore: H2D of each chunk's blobs -> staging[b], decode -> zraw, unpack+verify.
int tpi_restore_z(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total,
                  const void* host_src, const uint32_t* crcs, const uint32_t* csizes,
                  uint64_t signal_stream, uint64_t* bad_tiles, int64_t* first_bad,
                  tpi_stats* stats) {
  TpiRange range("tpi_restore_z");
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
  TpiRange range("tpi_restore_stream");
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

}  // extern "C"
