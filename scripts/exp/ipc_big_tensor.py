#!/usr/bin/env python3
"""HBM hand-off of a state that holds one tensor of ``--mib`` MiB (round 4).

``scripts/exp/ipc_lifetime.py`` found that ``hipIpcOpenMemHandle`` blocks on a PyTorch
allocation of 2 GiB or more (2040 MiB opens at once; 2048 and 2100 MiB block; one ``hipMalloc``
of 4 GiB opens at once).  This runs the production path on such a state: the predecessor
binds ``{"big": <mib MiB>, "small": 1 MiB}`` to a Checkpointer and exports it
(``export_hbm``); the successor checks ``hbm_ready`` and copies it (``restore_hbm``).
Timestamped phases on stderr; one JSON line on stdout.  Before ``IPC_MAX_ALLOC`` the 2560 MiB
case blocked in ``restore_hbm``; now the export is refused and the successor sees no hand-off.
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

EXPORTER = r'''
import sys, time, torch
sys.path.insert(0, %(root)r)
from terraform_provider_iterative_amd.checkpoint import Checkpointer, CheckpointError
g = torch.Generator(device="cuda").manual_seed(3)
t = {"big": torch.randn(%(n)d // 4, device="cuda", generator=g),
     "small": torch.randn(1 << 18, device="cuda", generator=g)}
ck = Checkpointer(t, path=%(path)r)
try:
    print("exported", ck.export_hbm(), flush=True)
except CheckpointError as error:  # IPC_MAX_ALLOC: the successor takes the host path
    print("refused", error, flush=True)
sys.stdin.readline()
'''

T0 = time.time()


def say(msg):
    print("[%.3f] successor: %s" % (time.time() - T0, msg), file=sys.stderr, flush=True)


def main():
    mib = float(sys.argv[sys.argv.index("--mib") + 1]) if "--mib" in sys.argv else 2560
    n = int(mib * (1 << 20)) // 4 * 4
    import torch

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    path = "/dev/shm/tpi-ipc-big-%d.spill" % os.getpid()
    child = subprocess.Popen([sys.executable, "-c", EXPORTER % {"root": ROOT, "n": n,
                                                                "path": path}],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        line = child.stdout.readline()
        assert line.startswith(("exported", "refused")), line
        say("predecessor: %s" % line.strip())
        g = torch.Generator(device="cuda").manual_seed(3)
        want = {"big": torch.randn(n // 4, device="cuda", generator=g),
                "small": torch.randn(1 << 18, device="cuda", generator=g)}
        dst = {k: torch.zeros_like(v) for k, v in want.items()}
        ck = Checkpointer(dst, path=path)
        out = {"mib": mib, "exporter": line.split()[0], "hbm_ready": ck.hbm_ready()}
        say("hbm_ready %s" % out["hbm_ready"])
        if out["hbm_ready"]:
            t = time.time()
            res = ck.restore_hbm()
            torch.cuda.synchronize()
            out["restore_hbm_s"] = round(time.time() - t, 3)
            out["bad_tiles"] = res.bad_tiles
            out["equal"] = all(torch.equal(dst[k], want[k]) for k in want)
            say("restored in %.3f s" % out["restore_hbm_s"])
        ck.close()
        print(json.dumps(out), flush=True)
    finally:
        child.stdin.write("\n")
        child.stdin.flush()
        child.wait(60)
        for p in (path, path + ".hbm", path + ".hbm.claim"):
            if os.path.exists(p):
                os.remove(p)


if __name__ == "__main__":
    main()
