"""Experiment: H2D straight from page-cache pages of a file (mmap + hipHostRegister ReadOnly)
vs pread into a pinned bounce buffer."""
import ctypes, mmap, os, time
import torch

GB = int(float(os.environ.get("GB", "4")) * 1e9)
path = os.environ.get("FILE", "/tmp/tpi-zc.bin")
with open(path, "wb") as f:
    blk = os.urandom(64 << 20)
    left = GB
    while left > 0:
        f.write(blk[:min(left, len(blk))]); left -= len(blk)
os.sync() if hasattr(os, "sync") else None
hip = ctypes.CDLL("libamdhip64.so")
torch.cuda.init()
dev = torch.empty(GB, dtype=torch.uint8, device="cuda")
stream = torch.cuda.Stream()
res = {}
for flags_name, flags in (("readonly", 0x08 | 0x02), ("readonly_pop", 0x08 | 0x02),
                          ("mapped_pop", 0x02)):
    ro = flags_name.startswith("readonly")
    fd = os.open(path, os.O_RDONLY if ro else os.O_RDWR)
    prot = mmap.PROT_READ if ro else mmap.PROT_READ | mmap.PROT_WRITE
    mflags = mmap.MAP_SHARED | (mmap.MAP_POPULATE if flags_name.endswith("_pop") else 0)
    t_map = time.perf_counter()
    m = mmap.mmap(fd, GB, mflags, prot)
    t_map = time.perf_counter() - t_map
    os.close(fd)
    addr = ctypes.addressof(ctypes.c_char.from_buffer(m)) if not ro else None
    if addr is None:
        buf = (ctypes.c_char * 1).from_buffer_copy(b"x")
        # read-only mapping: get its address through numpy
        import numpy as np
        a = np.frombuffer(m, dtype=np.uint8)
        addr = a.ctypes.data
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(ctypes.c_void_p(addr), ctypes.c_size_t(GB), ctypes.c_uint(flags))
    t1 = time.perf_counter()
    if rc != 0:
        res[flags_name] = {"register_rc": rc}
        continue
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    rc2 = hip.hipMemcpy(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(addr), ctypes.c_size_t(GB), 1)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    ok = bool(dev[:1024].cpu().numpy().tobytes() == open(path, "rb").read(1024))
    hip.hipHostUnregister(ctypes.c_void_p(addr))
    t4 = time.perf_counter()
    res[flags_name] = {"map_s": round(t_map, 4), "register_s": round(t1 - t0, 4), "h2d_GBps": round(GB / (t3 - t2) / 1e9, 2),
                       "memcpy_rc": rc2, "unregister_s": round(t4 - t3, 4), "ok": ok}
# bounce-buffer baseline
host = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
t0 = time.perf_counter()
with open(path, "rb", buffering=0) as f:
    off = 0
    while off < GB:
        n = f.readinto(memoryview(host.numpy())[:min(256 << 20, GB - off)])
        dev[off:off + n].copy_(host[:n])
        off += n
torch.cuda.synchronize()
res["bounce_serial_GBps"] = round(GB / (time.perf_counter() - t0) / 1e9, 2)
os.remove(path)
print(res)
