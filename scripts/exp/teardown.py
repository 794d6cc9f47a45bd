"""Experiment: what a 100 GB rank's exit and a successor's host-region setup cost."""
import json, os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
GB = float(os.environ.get("GB", "100"))
SHM = "/dev/shm/tpi-exp.region"

CHILD = r'''
import ctypes, os, sys, time
sys.path.insert(0, %(root)r)
import torch
from terraform_provider_iterative_amd.ops import hip
mode = sys.argv[1]; n = int(%(gb)r * 1e9)
lib = hip()
t = {}
if "gpu" in mode:
    t0 = time.time(); x = torch.empty(n, dtype=torch.uint8, device="cuda"); x.fill_(1); torch.cuda.synchronize(); t["gpu_alloc"] = time.time() - t0
if "host" in mode:
    populate = 0 if "nopop" in mode else 1
    t0 = time.time(); p = lib.tpi_host_map(%(shm)r.encode(), n, 0, populate); t["map"] = time.time() - t0
    t0 = time.time(); lib.check(lib.tpi_host_register(ctypes.c_void_p(p), n), "reg"); t["register"] = time.time() - t0
print(repr(t), flush=True)
os._exit(0)
'''

def run(mode):
    src = CHILD % {"root": ROOT, "gb": GB, "shm": SHM}
    t0 = time.time()
    p = subprocess.Popen([sys.executable, "-c", src, mode], stdout=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    t_line = time.time()
    p.wait()
    return {"mode": mode, "child": line.strip(), "exit_after_report_s": round(time.time() - t_line, 3),
            "total_s": round(time.time() - t0, 3)}

out = [run(m) for m in ("gpu", "host", "host", "host-nopop", "gpu+host")]
os.remove(SHM)
print(json.dumps(out, indent=1))
