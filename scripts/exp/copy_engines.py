"""Which engine moves a device<->pinned-host hipMemcpyAsync on this image?

    python scripts/exp/copy_engines.py <register|hostmalloc> <d2h|h2d> [GiB]

Run under ``rocprofv3 --kernel-trace --stats``: a blit-kernel copy shows up as
``__amd_rocclr_copyBuffer`` kernels, an SDMA copy as none.  Prints GB/s.
"""
import ctypes
import mmap
import sys
import time

import torch

kind, direction = sys.argv[1], sys.argv[2]
gib = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
n = int(gib * (1 << 30))
import os

hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
for name, args in (("hipHostRegister", [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]),
                   ("hipHostMalloc", [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                      ctypes.c_uint]),
                   ("hipMemcpyAsync", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_int, ctypes.c_void_p]),
                   ("hipStreamSynchronize", [ctypes.c_void_p])):
    getattr(hip, name).argtypes = args
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
dev.fill_(7)
torch.cuda.synchronize()
if kind == "register":
    m = mmap.mmap(-1, n)
    host = ctypes.addressof((ctypes.c_char * n).from_buffer(m))
    ctypes.memset(host, 1, n)
    assert hip.hipHostRegister(ctypes.c_void_p(host), n, 0x3) == 0
else:
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), n, 0) == 0
    host = p.value
    ctypes.memset(host, 1, n)
stream = torch.cuda.Stream()
s = ctypes.c_void_p(stream.cuda_stream)
dst, src, k = (host, dev.data_ptr(), 2) if direction == "d2h" else (dev.data_ptr(), host, 1)
for it in range(2):
    hip.hipMemcpyAsync(ctypes.c_void_p(dst), ctypes.c_void_p(src), n, k, s)
hip.hipStreamSynchronize(s)
reps = 8
t0 = time.perf_counter()
for it in range(reps):
    hip.hipMemcpyAsync(ctypes.c_void_p(dst), ctypes.c_void_p(src), n, k, s)
hip.hipStreamSynchronize(s)
dt = time.perf_counter() - t0
print("%s %s %.1f GB/s" % (kind, direction, reps * n / dt / 1e9), flush=True)
