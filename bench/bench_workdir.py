#!/usr/bin/env python3
"""Config 2: 1 x MI355X ``iterative_task`` with a large synthetic workdir + PyTorch-ROCm
``train.py`` (examples/train/train.py), driven through ``tpi apply``/``destroy`` like a user.

Reports apply -> first-log latency, workdir push GB/s (task storage), HBM staging GB/s
(by the runtime's stager before the rank starts, or ``--stage off``: by train.py itself),
training step time and the end-to-end wall time.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MAIN_TF = '''
resource "iterative_task" "train" {
  name    = "workdir-bench"
  cloud   = "%(cloud)s"
  machine = "%(machine)s"
  timeout = 3600
  environment = { TPI_FRAMEWORK_ROOT = "%(root)s", TPI_STAGE = "%(stage)s" }
  storage {
    workdir = "."
    output  = "results"
  }
  script = <<-END
    #!/bin/sh
    echo "task started on $TPI_MACHINE_IDENTITY"
    exec %(python)s %(root)s/examples/train/train.py --stage --steps %(steps)d
  END
}
'''


def make_workdir(path: str, total: int, files: int) -> None:
    block = os.urandom(64 << 20)
    per = total // files
    for i in range(files):
        with open(os.path.join(path, "shard-%03d.bin" % i), "wb") as handle:
            left = per
            handle.write(i.to_bytes(8, "little"))
            left -= 8
            while left > 0:
                n = min(left, len(block))
                handle.write(block[:n])
                left -= n


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gb", type=float, default=10.0)
    p.add_argument("--files", type=int, default=10)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--cloud", default="mi355x")
    p.add_argument("--machine", default="m+mi355x")
    p.add_argument("--base", default=None, help="scratch directory (default $TMPDIR)")
    p.add_argument("--stage", choices=("auto", "off"), default="auto",
                   help="auto: the runtime's stager puts the workdir in HBM before train.py "
                        "starts; off: train.py stages it itself (library path)")
    args = p.parse_args()
    base = tempfile.mkdtemp(prefix="tpi-workdir-", dir=args.base)
    try:
        work = os.path.join(base, "work")
        os.makedirs(work)
        total = int(args.gb * 1e9)
        free = shutil.disk_usage(base).free
        if free < 2.3 * total:
            raise SystemExit("need %.1f GB free in %s, have %.1f" % (2.3 * total / 1e9, base,
                                                                      free / 1e9))
        t = time.perf_counter()
        make_workdir(work, total, args.files)
        gen_s = time.perf_counter() - t
        with open(os.path.join(work, "main.tf"), "w") as handle:
            handle.write(MAIN_TF % {"cloud": args.cloud, "machine": args.machine, "root": ROOT,
                                    "python": sys.executable, "steps": args.steps,
                                    "stage": args.stage})
        env = dict(os.environ, TPI_STATE_ROOT=os.path.join(base, "state"))
        tpi = [sys.executable, os.path.join(ROOT, "bin", "tpi")]
        t0 = time.perf_counter()
        apply = subprocess.Popen(tpi + ["apply", "-auto-approve"], cwd=work, env=env,
                                 stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        pattern = os.path.join(base, "state", "*", "*", "reports", "task-*")
        first_log = None
        while first_log is None and time.perf_counter() - t0 < 600:
            for path in glob.glob(pattern):
                if os.path.getsize(path) > 0:
                    first_log = time.perf_counter() - t0
            time.sleep(0.001)
        out, _ = apply.communicate(timeout=600)
        apply_s = time.perf_counter() - t0
        logs = ""
        deadline = time.time() + 1800
        while time.time() < deadline:
            logs = "".join(open(p).read() for p in glob.glob(pattern))
            if "done {" in logs or "Traceback" in logs:
                break
            time.sleep(0.5)
        wall = time.perf_counter() - t0
        stats = {}
        m = re.search(r"done (\{.*\})", logs)
        if m:
            stats = json.loads(m.group(1))
        events = []
        for path in glob.glob(os.path.join(base, "state", "*", "*", "supervisor",
                                           "events.jsonl")):
            with open(path) as handle:
                events += [json.loads(line) for line in handle if line.strip()]
        pushed = next((e["description"] for e in events if e["code"] == "pushed"), None)
        staged = next((e for e in events if e["code"] == "workdir-staged"), None)
        started = next((e for e in events if e["code"] == "started"), None)
        d = subprocess.run(tpi + ["destroy", "-auto-approve"], cwd=work, env=env,
                           capture_output=True, text=True)
        result = {
            "config": "1xMI355X iterative_task: %.0f GB synthetic workdir sync + PyTorch-ROCm "
                      "train.py" % args.gb,
            "workdir_bytes": total, "files": args.files, "generate_s": round(gen_s, 2),
            "apply_to_first_log_s": round(first_log, 4) if first_log else None,
            "apply_s": round(apply_s, 3),
            "push_GBps": round(total / apply_s / 1e9, 2) if apply_s else None,
            "stage_GBps": stats.get("stage_GBps"), "train_step_ms": stats.get("step_ms"),
            "stage_stats": {k: stats.get(k) for k in ("attach_s", "load_ms", "read_ms",
                                                       "fanout_ms", "verify_ms", "load_GBps",
                                                       "staged_GBps", "verified", "load_s",
                                                       "read_s", "files")},
            "staging": "runtime (tpi-stager)" if args.stage == "auto" else "train.py",
            "end_to_end_s": round(wall, 2), "apply_ok": apply.returncode == 0,
            # the product's own journal: the push (reflinked or copied), the stager's load
            "push_s": float(pushed[2].split()[0]) if pushed else None,
            "push_method": pushed[3] if pushed else None,
            "stage_s": round(staged["time"] - started["time"], 3) if staged and started
            else None,
            "staged_event": staged["description"] if staged else None,
            "gpu_drain": [e["description"] for e in events if e["code"] == "gpu-drain"],
            "destroy_ok": d.returncode == 0,
        }
        if apply.returncode != 0 or not m:
            result["apply_output"] = out[-2000:]
            result["logs_tail"] = logs[-3000:]
        print(json.dumps(result))
    finally:
        shutil.rmtree(base, ignore_errors=True)


if __name__ == "__main__":
    main()
