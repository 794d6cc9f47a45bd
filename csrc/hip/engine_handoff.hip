// Device-to-device entry points of the engine (engine_internal.h): the HBM-to-HBM hand-off
// (allocation ranges, IPC export, the fused copy + read-back verify) and the device-side
// wrappers of the codec, hash, CRC and pack kernels.
#include "engine_internal.h"

using namespace tpi_engine_detail;

extern "C" {

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
  TpiRange range("tpi_copy_segments");
  std::lock_guard<std::mutex> lk(e->mu);
  auto t0 = std::chrono::steady_clock::now();
  if (check_segments(src, n, total)) return -1;
  bool fused = true;
  for (int i = 0; i < n && fused; ++i)
    fused = src[i].off == dst[i].off && src[i].nbytes == dst[i].nbytes;
  if (const char* m = getenv("TPI_HANDOFF_COPY")) fused = fused && strcmp(m, "staged") != 0;
  if (prepare(e, dst, n, total, !fused)) return -1;  // dst -> d_segs (+ staging if staged)
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

}  // extern "C"
