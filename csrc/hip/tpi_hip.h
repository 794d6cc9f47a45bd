// C ABI of libtpi_hip.so — the MI355X data plane of the task runtime.
//
// Hot paths replaced:
//   N2  workdir/checkpoint change detection  -> tpi_shard_hash   (XXH64-striped per shard)
//   N4  transparent checkpoint               -> tpi_save/tpi_restore (pack + CRC32C tiles,
//                                               pinned host spill on a side stream)
//   N1  workdir staging host -> HBM          -> tpi_h2d_chunks / pinned host mappings
//
// Everything here is plain C so the library can be loaded with ctypes after `import torch`
// (so it binds to the libamdhip64.so.7 torch already mapped) and linked by C++ tools.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TPI_MAX_DIMS 6
#define TPI_SEG_ALIGN 256  // packed-stream alignment of every tensor payload

// Segment kinds.  sizes/strides always describe the view (canonicalised: size-1 dims
// dropped, mergeable dims merged), so any kind may fall back to the element-wise path.
enum {
  TPI_SEG_CONTIG = 0,     // one contiguous run
  TPI_SEG_STRIDED = 1,    // general view: element gather/scatter
  TPI_SEG_ROWS = 2,       // last dim contiguous (sliced rows): 16-byte vector path
  TPI_SEG_TRANSPOSE = 3,  // (B,) R, C with R unit-stride: LDS-tiled transpose pre/post pass
};

// One tensor payload inside the packed checkpoint stream.
typedef struct tpi_seg {
  uint64_t ptr;     // device (or host-mapped) address of the tensor's first element
  uint64_t off;     // byte offset in the packed stream (multiple of TPI_SEG_ALIGN)
  uint64_t nbytes;  // payload bytes (numel * elem)
  uint32_t kind;    // TPI_SEG_*
  uint32_t elem;    // element size in bytes (strided path)
  int32_t ndim;
  int32_t pad_;
  int64_t sizes[TPI_MAX_DIMS];
  int64_t strides[TPI_MAX_DIMS];  // in elements
} tpi_seg;

enum { TPI_MODE_SDMA = 0, TPI_MODE_DIRECT = 1 };

// Stream arguments are hipStream_t values: 0 is the null (default) stream -- what torch's
// default stream is -- and TPI_NO_STREAM means "no ordering with any caller stream".
#define TPI_NO_STREAM (~0ull)

typedef struct tpi_engine tpi_engine;

typedef struct tpi_stats {
  double pack_ms;     // device time of pack/unpack kernels (sum)
  double copy_ms;     // wall time of the whole pipeline
  uint64_t bytes;     // packed bytes moved
  uint64_t chunks;
} tpi_stats;

// Bumped whenever a signature below changes (ops/_loader.py checks it).
#define TPI_ABI_VERSION 7

// Library / device
const char* tpi_last_error(void);
int tpi_version(void);                 // TPI_ABI_VERSION
const char* tpi_version_string(void);  // release version (_version.py)
int tpi_device_count(int* count);
int tpi_device_numa_node(int device, int* node);
int tpi_device_pci_bus_id(int device, char* buf, int len);

// Engine: per-device streams, staging ring, CRC tables.
tpi_engine* tpi_engine_create(int device, uint64_t chunk_bytes, int nbuf, uint64_t tile_bytes);
void tpi_engine_destroy(tpi_engine* e);
uint64_t tpi_engine_tile_bytes(const tpi_engine* e);
uint64_t tpi_engine_chunk_bytes(const tpi_engine* e);
// SDMA engine bit (hsa_amd_sdma_engine_id_t) that carries the engine's device -> host copies,
// 0 when they run as HIP blit kernels (TPI_D2H_ENGINE=blit or no engine available).
uint32_t tpi_engine_d2h_engine(const tpi_engine* e);
// Chunks whose H2D the last tpi_restore_stream split over two copy streams (it trailed the
// writer by TPI_H2D_SPLIT_LEAD chunks, default 2; "off" never splits).
uint64_t tpi_engine_split_chunks(const tpi_engine* e);

// Pack `segs` (n entries, sorted by off) into a stream of `total` bytes written to `host_dst`
// (pinned or host-mapped).  `crcs_out` (host, ceil(total/tile) entries) receives the CRC32C of
// every tile.  `wait_stream` (or TPI_NO_STREAM) is a stream whose prior work must finish first.
int tpi_save(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* host_dst,
             uint32_t* crcs_out, int mode, uint64_t wait_stream, tpi_stats* stats);
// Inverse: stream `total` bytes from `host_src`, verify each tile against `crcs`, scatter.
// `signal_stream` (or TPI_NO_STREAM): the unpack starts after that stream's pending work and the
// stream waits for the unpack before its later work.
// Returns 0 and sets *bad_tiles (0 = all verified) / *first_bad (-1 if none).
int tpi_restore(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total,
                const void* host_src, const uint32_t* crcs, int mode, uint64_t signal_stream,
                uint64_t* bad_tiles, int64_t* first_bad, tpi_stats* stats);

// Compressed (TPZ1, csrc/common/tpz.h) variants: the stream at `host_dst` is the concatenation
// of per-tile blobs whose sizes go to `csizes_out` (host, one u32 per tile; host_dst needs
// room for sum(tpz_bound(tile))).  *stream_bytes = bytes written.  CRCs cover the raw tiles.
int tpi_save_z(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* host_dst,
               uint32_t* crcs_out, uint32_t* csizes_out, uint64_t wait_stream,
               uint64_t* stream_bytes, tpi_stats* stats);
int tpi_restore_z(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total,
                  const void* host_src, const uint32_t* crcs, const uint32_t* csizes,
                  uint64_t signal_stream, uint64_t* bad_tiles, int64_t* first_bad,
                  tpi_stats* stats);
// Asynchronous checkpoints: (1) pack into a device snapshot buffer (`dev_dst`, `total`
// bytes; tile CRCs to `dev_crcs`), ordered after `wait_stream`'s work, with `wait_stream`
// made to wait for the pack -- the host is not blocked; (2) from any thread, spill the
// snapshot to `host_dst` (raw, or TPZ1-encoded when `codec` != 0, sizes to `csizes_out`)
// and its CRCs to `crcs_out`.  *stream_bytes = bytes written to host_dst.
int tpi_snapshot(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* dev_dst,
                 uint32_t* dev_crcs, uint64_t wait_stream);
int tpi_spill(tpi_engine* e, const void* dev_src, const uint32_t* dev_crcs, uint64_t total,
              void* host_dst, uint32_t* crcs_out, uint32_t* csizes_out, int codec,
              uint64_t* stream_bytes, tpi_stats* stats);
// Device-buffer codec (tests / tools): encode `len` bytes of `raw` into contiguous blobs
// (`meta_scratch`: ntiles*96 bytes, `csize`: ntiles u32), decode with blob offsets `coff`
// (ntiles+1 u64, device).
int tpi_tpz_encode_device(const void* raw, uint64_t len, uint64_t tile, void* meta_scratch,
                          uint32_t* csize, void* out, uint64_t stream);
int tpi_tpz_decode_device(const void* comp, const uint64_t* coff, uint64_t len, uint64_t tile,
                          void* raw, uint64_t stream);

// Incremental save: hash every tile of the packed stream straight from the tensors, compare
// with the digests of the previous sync (kept in the engine), and pack + spill only the tiles
// that changed into `host_dst` (stream offsets), updating their CRCs in `crcs_inout` (host,
// full array).  `full` forces every tile (first sync).  *dirty_tiles receives the count.
// `dev_prev` (device, ntiles u64, may be NULL = the engine's own): the digests the destination's
// content was written with; updated in place.
int tpi_sync(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total, void* host_dst,
             uint32_t* crcs_inout, uint64_t* dev_prev, int full, uint64_t wait_stream,
             uint64_t* dirty_tiles, tpi_stats* stats);
// Digest of every tile (device output, ntiles u64); exposed for tests.
int tpi_stream_hash(const tpi_seg* dev_segs, int n, uint64_t total, uint64_t tile_bytes,
                    uint64_t seed, uint64_t* dev_out, uint64_t stream);

// Device-buffer primitives (enqueued on `stream`, asynchronous).
int tpi_crc32c_tiles(const void* dev_ptr, uint64_t nbytes, uint64_t tile_bytes,
                     uint32_t* dev_out, uint64_t stream);
int tpi_shard_hash(const void* dev_ptr, uint64_t nbytes, uint64_t shard_bytes, uint64_t seed,
                   uint64_t* dev_out, uint64_t stream);
// Pack/unpack into/out of a device buffer (no host spill); used by tests and by the
// broadcast path (pack once, RCCL-broadcast the flat buffer, unpack on every rank).
// `host_segs` (may be NULL) is a host copy of the same descriptors: with it, transposed
// views go through the LDS-tiled transpose kernels instead of element gathers.
int tpi_pack_device(const tpi_seg* segs, const tpi_seg* host_segs, int n, uint64_t total,
                    void* dev_dst, uint64_t tile_bytes, uint32_t* dev_crcs, uint64_t stream);
int tpi_unpack_device(const tpi_seg* segs, const tpi_seg* host_segs, int n, uint64_t total,
                      void* dev_src, uint64_t tile_bytes, const uint32_t* dev_crcs,
                      uint64_t* dev_bad, uint64_t stream);

// Host memory: NUMA-bound, populated, registered (pinned) mappings.
// path == NULL -> anonymous; otherwise a shared file (e.g. /dev/shm/...) that outlives the
// process (the preemption spill target).  numa_node < 0 -> no binding.
void* tpi_host_map(const char* path, uint64_t bytes, int numa_node, int populate);
int tpi_host_unmap(void* ptr, uint64_t bytes);
int tpi_host_register(void* ptr, uint64_t bytes);
int tpi_host_unregister(void* ptr);
// Read-only registration of an existing (e.g. page-cache file) mapping for DMA reads: the
// zero-copy workdir staging path (runtime/workdir.py).  Populate the mapping first.
int tpi_host_register_ro(void* ptr, uint64_t bytes);
// Progressive pinning of an existing mapping (e.g. a preempted rank's spill file): pages are
// read-faulted by `threads` workers and hipHostRegister-ed window by window in background
// threads; tpi_host_pin_ready() is the registered prefix in bytes.  Release unregisters.
typedef struct tpi_pinner tpi_pinner;
tpi_pinner* tpi_host_pin_start(void* base, uint64_t bytes, uint64_t window, int threads);
uint64_t tpi_host_pin_ready(const tpi_pinner* p);
// hold != 0: register no further window until released, or until a copy waits for one
int tpi_host_pin_hold(tpi_pinner* p, int hold);
uint64_t tpi_host_pin_window(const tpi_pinner* p);
int tpi_host_pin_wait(tpi_pinner* p);
int tpi_host_pin_release(tpi_pinner* p);
// The engine's host region is registered per `window` (pinner may be NULL once complete): its
// copies are split at window boundaries and wait for their window (restore overlaps pinning).
// Only the staged (sdma) pipelines support such a region.
// Streaming hand-off (preemption).  While `words` is set, tpi_save / tpi_save_z publish into
// it (host memory shared with the successor process) after each chunk's device -> host copy:
// words[1] = stream bytes in host memory, then words[0] = tiles whose bytes and CRCs (and
// blob sizes) are there, both release-stored.  NULL stops publishing.
int tpi_engine_set_progress(tpi_engine* e, uint64_t* words);
// Streamed restores (tpi_restore_stream[_at]) copy host -> device on an SDMA engine of their
// own, driven from the host (on != 0), instead of hipMemcpyAsync.  Returns the engine index,
// or -1 when no engine is free (the restores then keep hipMemcpyAsync).
int tpi_engine_set_h2d_sdma(tpi_engine* e, int on);
// Allocate the buffers the pipelines would otherwise allocate on first use, for up to
// `nsegs` segments and `ntiles` tiles (and the codec's decode buffers when `codec`).
int tpi_engine_reserve(tpi_engine* e, int nsegs, uint64_t ntiles, int codec);
// Allocate the engine's HBM staging ring now (engines allocate it at their first pipeline
// that moves data through it; the HBM hand-off copy never does).
int tpi_engine_alloc_staging(tpi_engine* e);
// Restore while another process is still writing the region: chunk k is copied once words[0]
// covers its tiles; `timeout_s` without progress fails the call.  csizes == NULL: raw stream.
int tpi_restore_stream(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total,
                       const void* host_src, const uint32_t* crcs, const uint32_t* csizes,
                       const uint64_t* words, double timeout_s, uint64_t signal_stream,
                       uint64_t* bad_tiles, int64_t* first_bad, tpi_stats* stats);
// tpi_restore_stream of a stretch of the writer's stream that starts at its tile `tile_base`
// (segs/total/host_src/crcs/csizes describe the stretch; words count the whole stream).
int tpi_restore_stream_at(tpi_engine* e, const tpi_seg* segs, int n, uint64_t total,
                          const void* host_src, const uint32_t* crcs, const uint32_t* csizes,
                          const uint64_t* words, uint64_t tile_base, double timeout_s,
                          uint64_t signal_stream, uint64_t* bad_tiles, int64_t* first_bad,
                          tpi_stats* stats);
// HBM-to-HBM hand-off between processes on one GPU.  tpi_ipc_export: IPC handle
// (TPI_IPC_HANDLE_BYTES) of the allocation holding `ptr` -- e.g. inside a torch caching-
// allocator segment -- and ptr's offset in it; the successor maps it with tpi_ipc_open.
// tpi_copy_segments moves tensors described by `src` (e.g. a predecessor's, mapped over IPC)
// into `dst` through the pack / unpack kernels, tile CRCs verified (`bad_tiles`); both plans
// must describe the same stream.
// Base address and size of the device allocation holding ptr (exporters call
// tpi_ipc_export once per allocation, not once per tensor).
int tpi_mem_range(const void* ptr, uint64_t* base_out, uint64_t* alloc_bytes_out);
int tpi_ipc_export(const void* ptr, void* handle_out, uint64_t* offset_out,
                   uint64_t* alloc_bytes_out);
int tpi_copy_segments(tpi_engine* e, const tpi_seg* src, const tpi_seg* dst, int n,
                      uint64_t total, uint64_t signal_stream, uint64_t* bad_tiles,
                      tpi_stats* stats);
// The hand-off's default route (sdma.cpp): an allocation as a dma-buf file descriptor (any
// size; `offset_out` = ptr's offset in the buffer), mapped by another process into its GPU
// address space (tpi_dmabuf_import: base and size of the mapping) and unmapped again.
int tpi_dmabuf_available(void);
int tpi_dmabuf_export(const void* ptr, uint64_t size, int* fd_out, uint64_t* offset_out);
int tpi_dmabuf_close(int fd);
int tpi_dmabuf_import(int device, int fd, void** ptr_out, uint64_t* size_out);
int tpi_dmabuf_unmap(void* ptr);
// Plain device allocations (hipMalloc / hipFree) and a synchronous device-to-device copy.
int tpi_dev_alloc(uint64_t bytes, void** out);
int tpi_dev_free(void* ptr);
int tpi_d2d(void* dst, const void* src, uint64_t bytes, uint64_t stream);
int tpi_engine_set_host_region(tpi_engine* e, void* base, uint64_t bytes, uint64_t window,
                               tpi_pinner* pinner);
// hipMemcpyAsync host -> device on `stream` (0 = legacy default stream).
int tpi_h2d_async(void* dev_dst, const void* host_src, uint64_t bytes, uint64_t stream);

// Chunked host->device copy through the engine's copy stream (workdir staging).
int tpi_h2d(tpi_engine* e, void* dev_dst, const void* host_src, uint64_t bytes);
int tpi_d2h(tpi_engine* e, void* host_dst, const void* dev_src, uint64_t bytes);

// ---- Workdir staging (N1): host files <-> a flat image (runtime/stage.py) ---------------------
// Bytes [0, size) of `path` live at image offset `offset`; files sorted by offset, disjoint.
typedef struct tpi_file {
  const char* path;
  uint64_t offset;
  uint64_t size;
} tpi_file;
typedef struct tpi_loader tpi_loader;
// device >= 0: the image is device memory, filled through a pinned ring of `nbuf` chunks of
// `chunk_bytes` (NUMA node `numa_node`, < 0 = unbound) on the loader's copy stream; device < 0:
// the image is host memory.  `threads` pread workers per chunk.
tpi_loader* tpi_loader_create(int device, uint64_t chunk_bytes, int nbuf, int threads,
                              int numa_node);
void tpi_loader_destroy(tpi_loader* L);
// Fill image bytes [lo, hi) of `dst` (image base) from the files; bytes no file covers are 0.
// stats: copy_ms = wall, pack_ms = host read time, bytes, chunks.
int tpi_loader_load(tpi_loader* L, const tpi_file* files, uint64_t nfiles, uint64_t lo,
                    uint64_t hi, void* dst, tpi_stats* stats);
// Write image ranges ([lo, hi) pairs, `nranges` of them) of `src` back into the files.
int tpi_loader_store(tpi_loader* L, const tpi_file* files, uint64_t nfiles,
                     const uint64_t* ranges, uint64_t nranges, const void* src,
                     tpi_stats* stats);

// ---- HIP IPC: a staged image mapped zero-copy by the rank processes ------------------------
#define TPI_IPC_HANDLE_BYTES 64
int tpi_ipc_handle(void* dev_ptr, uint8_t* out);
int tpi_ipc_open(const uint8_t* handle, int device, void** out);
int tpi_ipc_close(void* dev_ptr);

// ---- Task communicator (RCCL over xGMI) ------------------------------------
#define TPI_COMM_ID_BYTES 128
typedef struct tpi_comm tpi_comm;
int tpi_comm_unique_id(uint8_t* out);  // ncclGetUniqueId (rank 0 / the supervisor side)
tpi_comm* tpi_comm_init_rank(const uint8_t* id, int nranks, int rank, int device);
// One process driving `ndev` GPUs (the stager): out[i] = communicator of rank i on devices[i].
int tpi_comm_init_all(int ndev, const int* devices, tpi_comm** out);
void tpi_comm_destroy(tpi_comm* c);
int tpi_comm_rank(const tpi_comm* c);
int tpi_comm_size(const tpi_comm* c);
// Collectives over the `n` communicators this thread drives (1 in a rank process, all of
// them in a single-process stager), issued as one RCCL group on each communicator's own
// stream; `sync` waits for completion.
// In-place all-gather: rank r's shard sits at bufs[i] + r * shard_bytes.
int tpi_comm_allgather_inplace(tpi_comm** comms, int n, void** bufs, uint64_t shard_bytes,
                               int sync);
int tpi_comm_broadcast(tpi_comm** comms, int n, void** bufs, uint64_t bytes, int root, int sync);
int tpi_comm_sync(tpi_comm** comms, int n);
// NCCL groups this library has started and not ended (0 outside a collective call, also after
// a failed one); TPI_NCCL_FAIL_AT=<i> makes the i-th enqueue of a grouped collective fail.
int tpi_nccl_groups_open(void);

#ifdef __cplusplus
}
#endif
