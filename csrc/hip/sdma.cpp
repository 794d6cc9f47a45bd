// Device -> host copies on the GPU's SDMA copy engines.
//
// On this ROCm image hipMemcpyAsync D2H into pinned host memory runs as
// __amd_rocclr_copyBuffer blit kernels (128 workgroups x 1024 lanes for the whole copy), so a
// save's PCIe traffic occupies CUs next to the pack / CRC / TPZ1 kernels and stretches them
// (profiles/rocprof_headline_100g_round1.md).  H2D already goes to an SDMA engine.  Measured on
// MI355X (profiles/sdma_engines_round2.md): each of SDMA engines 0-3 moves D2H at 57 GB/s -- the
// same as the blit kernels, i.e. the PCIe Gen5 x16 wire -- so the copy can leave the CUs at no
// cost in bandwidth.
//
// The copies are issued with hsa_amd_memory_async_copy_on_engine() on the highest of the
// runtime's preferred D2H engines.  HSA is reached through the runtime HIP itself loaded (found with
// dl_iterate_phdr, bound with dlsym): torch ships its own libhsa-runtime64, and a second HSA
// runtime in the process must never be mapped.  Ordering with HIP streams is host-side: the
// pipelines wait for the producing kernel's event before issuing a copy, and wait for the
// lane's signal before a staging buffer is written again.
//
// TPI_D2H_ENGINE=blit keeps hipMemcpyAsync (A/B); the lanes are also off when HSA cannot be
// bound or the device has no SDMA engine to the host.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <link.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "internal.h"

namespace {

struct Hsa {
  bool ok = false;
  decltype(&hsa_init) init = nullptr;
  decltype(&hsa_iterate_agents) iterate_agents = nullptr;
  decltype(&hsa_agent_get_info) agent_get_info = nullptr;
  decltype(&hsa_status_string) status_string = nullptr;
  decltype(&hsa_signal_create) signal_create = nullptr;
  decltype(&hsa_signal_destroy) signal_destroy = nullptr;
  decltype(&hsa_signal_add_relaxed) signal_add = nullptr;
  decltype(&hsa_signal_load_scacquire) signal_load = nullptr;
  decltype(&hsa_signal_wait_scacquire) signal_wait = nullptr;
  decltype(&hsa_amd_memory_copy_engine_status) engine_status = nullptr;
  decltype(&hsa_amd_memory_get_preferred_copy_engine) preferred_engine = nullptr;
  decltype(&hsa_amd_memory_async_copy_on_engine) copy_on_engine = nullptr;
  // dma-buf hand-off (optional: absent symbols only disable that route)
  decltype(&hsa_amd_portable_export_dmabuf) export_dmabuf = nullptr;
  decltype(&hsa_amd_portable_close_dmabuf) close_dmabuf = nullptr;
  decltype(&hsa_amd_interop_map_buffer) interop_map = nullptr;
  decltype(&hsa_amd_interop_unmap_buffer) interop_unmap = nullptr;
};

int find_hsa(struct dl_phdr_info* info, size_t, void* data) {
  std::string* path = (std::string*)data;
  if (info->dlpi_name && strstr(info->dlpi_name, "libhsa-runtime64")) {
    *path = info->dlpi_name;
    return 1;
  }
  return 0;
}

const Hsa& hsa() {
  static Hsa h;
  static std::once_flag once;
  std::call_once(once, [] {
    // HIP must be up first, so that the HSA runtime in the process is the one it loaded.
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return;
    std::string path;
    dl_iterate_phdr(find_hsa, &path);
    if (path.empty()) return;
    void* lib = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (!lib) return;
#define BIND(field, sym)                                     \
  h.field = (decltype(h.field))dlsym(lib, #sym);             \
  if (!h.field) return;
    BIND(init, hsa_init);
    BIND(iterate_agents, hsa_iterate_agents);
    BIND(agent_get_info, hsa_agent_get_info);
    BIND(status_string, hsa_status_string);
    BIND(signal_create, hsa_signal_create);
    BIND(signal_destroy, hsa_signal_destroy);
    BIND(signal_add, hsa_signal_add_relaxed);
    BIND(signal_load, hsa_signal_load_scacquire);
    BIND(signal_wait, hsa_signal_wait_scacquire);
    BIND(engine_status, hsa_amd_memory_copy_engine_status);
    BIND(preferred_engine, hsa_amd_memory_get_preferred_copy_engine);
    BIND(copy_on_engine, hsa_amd_memory_async_copy_on_engine);
#undef BIND
    h.export_dmabuf = (decltype(h.export_dmabuf))dlsym(lib, "hsa_amd_portable_export_dmabuf");
    h.close_dmabuf = (decltype(h.close_dmabuf))dlsym(lib, "hsa_amd_portable_close_dmabuf");
    h.interop_map = (decltype(h.interop_map))dlsym(lib, "hsa_amd_interop_map_buffer");
    h.interop_unmap = (decltype(h.interop_unmap))dlsym(lib, "hsa_amd_interop_unmap_buffer");
    // Reference-counted: HIP already initialised the runtime, this only keeps it alive for
    // as long as we hold signals.
    h.ok = h.init() == HSA_STATUS_SUCCESS;
  });
  return h;
}

struct AgentQuery {
  uint32_t bdf = 0, domain = 0;
  hsa_agent_t gpu{}, cpu{};
  bool found = false;
};

hsa_status_t match_agent(hsa_agent_t a, void* data) {
  AgentQuery* q = (AgentQuery*)data;
  const Hsa& h = hsa();
  hsa_device_type_t type;
  if (h.agent_get_info(a, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS ||
      type != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, domain = 0;
  h.agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
  h.agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &domain);
  if (bdf != q->bdf || domain != q->domain) return HSA_STATUS_SUCCESS;
  if (h.agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NEAREST_CPU, &q->cpu) !=
      HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  q->gpu = a;
  q->found = true;
  return HSA_STATUS_INFO_BREAK;
}

std::string hsa_error(hsa_status_t s) {
  const char* m = nullptr;
  hsa().status_string(s, &m);
  return m ? m : ("HSA status " + std::to_string((int)s));
}

}  // namespace

struct tpi_sdma {
  hsa_agent_t gpu{}, cpu{};
  uint32_t engine = 0;                          // hsa_amd_sdma_engine_id_t bit
  std::vector<std::vector<hsa_signal_t>> lanes;  // signals of the copies in flight, per lane
  std::vector<hsa_signal_t> pool;               // completed signals, reused
};

namespace {

// One signal per copy (value 1, decremented by the engine): profilers that wrap the completion
// signal (rocprofv3 --memory-copy-trace) assume exactly that.
int take_signal(tpi_sdma* s, hsa_signal_t* out) {
  if (!s->pool.empty()) {
    *out = s->pool.back();
    s->pool.pop_back();
    hsa().signal_add(*out, 1);
    return 0;
  }
  hsa_status_t st = hsa().signal_create(1, 0, nullptr, out);
  if (st != HSA_STATUS_SUCCESS) return tpi_fail("hsa_signal_create: " + hsa_error(st));
  return 0;
}

}  // namespace

tpi_sdma* tpi_sdma_open(int device, int lanes) {
  const char* env = getenv("TPI_D2H_ENGINE");
  if (env && strcmp(env, "blit") == 0) return nullptr;
  const Hsa& h = hsa();
  if (!h.ok) return nullptr;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return nullptr;
  AgentQuery q;
  q.bdf = (uint32_t)((p.pciBusID << 8) | (p.pciDeviceID << 3));
  q.domain = (uint32_t)p.pciDomainID;
  h.iterate_agents(match_agent, &q);
  if (!q.found) return nullptr;
  uint32_t avail = 0, pref = 0, h2d = 0;
  if (h.engine_status(q.cpu, q.gpu, &avail) != HSA_STATUS_SUCCESS || !avail) return nullptr;
  if (h.preferred_engine(q.cpu, q.gpu, &pref) != HSA_STATUS_SUCCESS) pref = 0;
  if (h.preferred_engine(q.gpu, q.cpu, &h2d) != HSA_STATUS_SUCCESS) h2d = 0;
  // Candidates: the runtime's preferred D2H engines, or -- when the runtime has no preference
  // to report (torch's bundled HSA) -- engines 1-3, the host-facing engines next to engine 0
  // (MI355X: 57 GB/s D2H each; engines 4+ serve xGMI at 7-13 GB/s, sdma_engines_round2.md).
  // Never the engine HIP's H2D copies run on (preferred H2D, else engine 0): a restore that
  // streams in while a save streams out (preemption hand-off) shared engine 0 with them and
  // both directions fell to ~33 GB/s; on engine 2 they run side by side.
  uint32_t pick = (pref & avail) ? (pref & avail) : (avail & 0xEu);
  pick &= ~(h2d ? h2d : 0x1u);
  if (!pick) pick = avail;
  tpi_sdma* s = new tpi_sdma();
  s->gpu = q.gpu;
  s->cpu = q.cpu;
  s->engine = 1u << (31 - __builtin_clz(pick));  // highest candidate
  if (env && strncmp(env, "sdma", 4) == 0 && env[4]) {  // TPI_D2H_ENGINE=sdma<i>: that engine
    const int id = atoi(env + 4);
    if (id >= 0 && id < 16 && (avail & (1u << id))) s->engine = 1u << id;
  }
  s->lanes.resize(lanes > 0 ? lanes : 1);
  return s;
}

// Host -> device lanes for a restore that must keep off the engines the runtime uses: the
// H2D engine HIP itself would pick (preferred H2D, else engine 0, which the kernel driver's
// own buffer clears share) and the D2H engine tpi_sdma_open picks for saves.
// TPI_H2D_ENGINE=sdma<i> pins an engine.  nullptr when no such engine is free.
tpi_sdma* tpi_sdma_open_h2d(int device, int lanes) {
  const Hsa& h = hsa();
  if (!h.ok) return nullptr;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return nullptr;
  AgentQuery q;
  q.bdf = (uint32_t)((p.pciBusID << 8) | (p.pciDeviceID << 3));
  q.domain = (uint32_t)p.pciDomainID;
  h.iterate_agents(match_agent, &q);
  if (!q.found) return nullptr;
  uint32_t avail = 0, pref = 0, h2d = 0;
  if (h.engine_status(q.gpu, q.cpu, &avail) != HSA_STATUS_SUCCESS || !avail) return nullptr;
  if (h.preferred_engine(q.cpu, q.gpu, &pref) != HSA_STATUS_SUCCESS) pref = 0;
  if (h.preferred_engine(q.gpu, q.cpu, &h2d) != HSA_STATUS_SUCCESS) h2d = 0;
  uint32_t d2h_pick = (pref & avail) ? (pref & avail) : (avail & 0xEu);
  d2h_pick &= ~(h2d ? h2d : 0x1u);
  const uint32_t d2h = d2h_pick ? 1u << (31 - __builtin_clz(d2h_pick)) : 0;
  uint32_t pick = avail & 0xEu & ~(h2d ? h2d : 0x1u) & ~d2h;  // host-facing engines 1-3
  uint32_t engine = pick ? (pick & (~pick + 1)) : 0;         // lowest candidate
  const char* env = getenv("TPI_H2D_ENGINE");
  if (env && strncmp(env, "sdma", 4) == 0 && env[4]) {
    const int id = atoi(env + 4);
    if (id >= 0 && id < 16 && (avail & (1u << id))) engine = 1u << id;
  }
  if (!engine) return nullptr;
  tpi_sdma* s = new tpi_sdma();
  s->gpu = q.gpu;
  s->cpu = q.cpu;
  s->engine = engine;
  s->lanes.resize(lanes > 0 ? lanes : 1);
  return s;
}

int tpi_sdma_h2d(tpi_sdma* s, int lane, void* dev_dst, const void* host_src, size_t n) {
  if (!n) return 0;
  hsa_signal_t sig;
  if (take_signal(s, &sig)) return -1;
  hsa_status_t st = hsa().copy_on_engine(dev_dst, s->gpu, host_src, s->cpu, n, 0, nullptr, sig,
                                         (hsa_amd_sdma_engine_id_t)s->engine, true);
  if (st != HSA_STATUS_SUCCESS) {
    hsa().signal_add(sig, -1);
    s->pool.push_back(sig);
    return tpi_fail("hsa_amd_memory_async_copy_on_engine (H2D): " + hsa_error(st));
  }
  s->lanes[lane % s->lanes.size()].push_back(sig);
  return 0;
}

void tpi_sdma_close(tpi_sdma* s) {
  if (!s) return;
  tpi_sdma_wait_all(s);
  for (hsa_signal_t sig : s->pool) hsa().signal_destroy(sig);
  delete s;
}

uint32_t tpi_sdma_engine(const tpi_sdma* s) { return s ? s->engine : 0; }

int tpi_sdma_d2h(tpi_sdma* s, int lane, void* host_dst, const void* dev_src, size_t n) {
  if (!n) return 0;
  hsa_signal_t sig;
  if (take_signal(s, &sig)) return -1;
  hsa_status_t st = hsa().copy_on_engine(host_dst, s->cpu, dev_src, s->gpu, n, 0, nullptr, sig,
                                         (hsa_amd_sdma_engine_id_t)s->engine, true);
  if (st != HSA_STATUS_SUCCESS) {
    hsa().signal_add(sig, -1);
    s->pool.push_back(sig);
    return tpi_fail("hsa_amd_memory_async_copy_on_engine: " + hsa_error(st));
  }
  s->lanes[lane % s->lanes.size()].push_back(sig);
  return 0;
}

int tpi_sdma_wait(tpi_sdma* s, int lane) {
  const Hsa& h = hsa();
  int rc = 0;
  auto& pending = s->lanes[lane % s->lanes.size()];
  for (hsa_signal_t sig : pending) {
    hsa_signal_value_t v;
    while ((v = h.signal_wait(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                              HSA_WAIT_STATE_BLOCKED)) > 0) {
    }
    if (v < 0) {  // the runtime reports a failed copy by driving the signal negative
      h.signal_add(sig, -v);
      rc = tpi_fail("SDMA copy failed (signal " + std::to_string((long long)v) + ")");
    }
    s->pool.push_back(sig);
  }
  pending.clear();
  return rc;
}

int tpi_sdma_wait_all(tpi_sdma* s) {
  int rc = 0;
  for (size_t i = 0; i < s->lanes.size(); ++i)
    if (tpi_sdma_wait(s, (int)i)) rc = -1;
  return rc;
}

// ---- HBM hand-off over dma-buf ------------------------------------------------------------
// hipIpcOpenMemHandle never returns for allocations of 2 GiB or more on this stack (round 5,
// profiles/round5/ipc_cause.md: the importer spins at 100 % CPU while the exporter's IPC
// server thread still waits in accept(); plain hipMalloc and PyTorch blocks alike).  The
// hand-off therefore moves its allocations as dma-buf file descriptors: the predecessor
// exports each allocation (DRM PRIME, any size), passes the descriptors over a Unix socket
// (SCM_RIGHTS, checkpoint/checkpointer.py), and the successor maps them into its own GPU
// address space with hsa_amd_interop_map_buffer.  A mapping holds its own reference to the
// memory, so it stays valid whatever the exporter does.

namespace {

bool device_agent(int device, hsa_agent_t* out) {
  static std::mutex mu;
  static std::vector<std::pair<int, hsa_agent_t>> cache;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& c : cache)
    if (c.first == device) {
      *out = c.second;
      return true;
    }
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess) return false;
  AgentQuery q;
  q.bdf = (uint32_t)((p.pciBusID << 8) | (p.pciDeviceID << 3));
  q.domain = (uint32_t)p.pciDomainID;
  hsa().iterate_agents(match_agent, &q);
  if (!q.found) return false;
  cache.push_back({device, q.gpu});
  *out = q.gpu;
  return true;
}

}  // namespace

extern "C" {

int tpi_dmabuf_available() {
  const Hsa& h = hsa();
  return h.ok && h.export_dmabuf && h.close_dmabuf && h.interop_map && h.interop_unmap;
}

int tpi_dmabuf_export(const void* ptr, uint64_t size, int* fd_out, uint64_t* offset_out) {
  if (!tpi_dmabuf_available()) return tpi_fail("dma-buf export: HSA entry points unavailable");
  int fd = -1;
  uint64_t off = 0;
  hsa_status_t st = hsa().export_dmabuf(ptr, (size_t)size, &fd, &off);
  if (st != HSA_STATUS_SUCCESS) return tpi_fail("hsa_amd_portable_export_dmabuf: " + hsa_error(st));
  *fd_out = fd;
  *offset_out = off;
  return 0;
}

int tpi_dmabuf_close(int fd) {
  if (!tpi_dmabuf_available()) return tpi_fail("dma-buf close: HSA entry points unavailable");
  hsa_status_t st = hsa().close_dmabuf(fd);
  if (st != HSA_STATUS_SUCCESS) return tpi_fail("hsa_amd_portable_close_dmabuf: " + hsa_error(st));
  return 0;
}

int tpi_dmabuf_import(int device, int fd, void** ptr_out, uint64_t* size_out) {
  if (!tpi_dmabuf_available()) return tpi_fail("dma-buf import: HSA entry points unavailable");
  hsa_agent_t agent;
  if (!device_agent(device, &agent)) return tpi_fail("dma-buf import: no HSA agent for device");
  size_t size = 0;
  void* ptr = nullptr;
  hsa_handle_t handle = fd;  // Linux: the dma-buf file descriptor itself
  hsa_status_t st = hsa().interop_map(1, &agent, handle, 0, &size, &ptr, nullptr, nullptr);
  if (st != HSA_STATUS_SUCCESS) return tpi_fail("hsa_amd_interop_map_buffer: " + hsa_error(st));
  *ptr_out = ptr;
  *size_out = size;
  return 0;
}

int tpi_dmabuf_unmap(void* ptr) {
  if (!tpi_dmabuf_available()) return tpi_fail("dma-buf unmap: HSA entry points unavailable");
  hsa_status_t st = hsa().interop_unmap(ptr);
  if (st != HSA_STATUS_SUCCESS) return tpi_fail("hsa_amd_interop_unmap_buffer: " + hsa_error(st));
  return 0;
}

}  // extern "C"
