#!/usr/bin/env python3
"""Does the dma-buf route move allocations that hipIpcOpenMemHandle cannot (>= 2 GiB)? (round 5)

One exporter and one importer, siblings under a driver that never touches the GPU (like a
preempted rank and its successor under the supervisor).  The exporter allocates ``--mib`` MiB
(PyTorch's caching allocator, or one hipMalloc with ``--raw``), fills it with a pattern, exports
it with ``tpi_dmabuf_export`` and passes the descriptor over a Unix socket (SCM_RIGHTS).  The
importer maps it with ``tpi_dmabuf_import``, checks the pattern with a kernel (a sum), unmaps it
and reports the timings.  The exporter stays alive until the importer is done (the importer never
reads after the exporter has exited).
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

EXPORTER = r'''
import ctypes, json, os, socket, sys, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.ops import hip
from terraform_provider_iterative_amd.runtime.stage import _device_tensor
n, raw = %(n)d, %(raw)r
sock = socket.socket(fileno=%(fd)d)
if raw:
    rt = ctypes.CDLL("libamdhip64.so")
    p = ctypes.c_void_p()
    assert rt.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)) == 0
    t = _device_tensor(p.value, n, 0).view(torch.int32)
else:
    t = torch.empty(n // 4, dtype=torch.int32, device="cuda")
t.copy_(torch.arange(n // 4, dtype=torch.int32, device="cuda") * 3 + 1)
torch.cuda.synchronize()
want = int(t.to(torch.int64).sum().item())
lib = hip()
fd, off = ctypes.c_int(-1), ctypes.c_uint64(0)
t0 = time.perf_counter()
lib.check(lib.tpi_dmabuf_export(ctypes.c_void_p(t.data_ptr()), n, ctypes.byref(fd),
                                ctypes.byref(off)), "export")
export_s = time.perf_counter() - t0
socket.send_fds(sock, [json.dumps({"sum": want, "offset": off.value, "n": n,
                                   "export_s": export_s}).encode()], [fd.value])
os.close(fd.value)
sock.recv(16)  # the importer is done
os._exit(0)
'''

IMPORTER = r'''
import ctypes, json, os, socket, sys, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.ops import hip
from terraform_provider_iterative_amd.runtime.stage import _device_tensor
lib = hip()
torch.empty(1, device="cuda"); torch.cuda.synchronize()
sock = socket.socket(fileno=%(fd)d)
msg, fds, _, _ = socket.recv_fds(sock, 4096, 4)
info = json.loads(msg)
ptr, size = ctypes.c_void_p(), ctypes.c_uint64(0)
t0 = time.perf_counter()
lib.check(lib.tpi_dmabuf_import(0, fds[0], ctypes.byref(ptr), ctypes.byref(size)), "import")
import_s = time.perf_counter() - t0
os.close(fds[0])
t = _device_tensor(ptr.value + info["offset"], info["n"], 0).view(torch.int32)
got = int(t.to(torch.int64).sum().item())
del t
torch.cuda.synchronize()
t0 = time.perf_counter()
lib.check(lib.tpi_dmabuf_unmap(ptr), "unmap")
unmap_s = time.perf_counter() - t0
print(json.dumps({"ok": got == info["sum"], "mapped_bytes": size.value, "offset": info["offset"],
                  "export_s": round(info["export_s"], 5), "import_s": round(import_s, 5),
                  "unmap_s": round(unmap_s, 5)}), flush=True)
sock.send(b"done")
'''


def main():
    mib = float(sys.argv[sys.argv.index("--mib") + 1]) if "--mib" in sys.argv else 2100
    raw = "--raw" in sys.argv
    n = int(mib * (1 << 20)) // 4 * 4
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    exp = subprocess.Popen([sys.executable, "-c", EXPORTER % {"root": ROOT, "n": n, "raw": raw,
                                                              "fd": a.fileno()}],
                           pass_fds=(a.fileno(),))
    imp = subprocess.Popen([sys.executable, "-c", IMPORTER % {"root": ROOT, "fd": b.fileno()}],
                           pass_fds=(b.fileno(),), stdout=subprocess.PIPE, text=True)
    a.close()
    b.close()
    t0 = time.time()
    out, _ = imp.communicate(timeout=90)
    exp.wait(30)
    rec = {"mib": mib, "allocator": "hipMalloc" if raw else "torch",
           "importer_rc": imp.returncode, "exporter_rc": exp.returncode,
           "wall_s": round(time.time() - t0, 2)}
    lines = [l for l in out.splitlines() if l.startswith("{")]
    if lines:
        rec.update(json.loads(lines[-1]))
    print(json.dumps(rec), flush=True)
    sys.exit(0 if rec.get("ok") else 1)


if __name__ == "__main__":
    main()
