"""Experiment: what a background checkpoint spill (Checkpointer.save_async) costs a training
loop running next to it on the same GPU.

A bf16 GEMM loop stands in for training.  The script measures its TFLOP/s alone, then while
a save_async spill of the synthetic AdamW state runs (TPZ1 codec on the engine's streams),
and reports the spill time with and without the GEMMs.

    python scripts/exp/async_interference.py [GB] [gemm_n] [chunk_MiB] [codec]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import synthetic_checkpoint  # noqa: E402
from terraform_provider_iterative_amd.checkpoint import Checkpointer  # noqa: E402


def gemm_rate(a, b, seconds, stop=None):
    """TFLOP/s of back-to-back a @ b for `seconds` (or until stop() is true)."""
    n = a.shape[0]
    done, t0 = 0, time.perf_counter()
    while True:
        for _ in range(8):
            torch.mm(a, b)
        torch.cuda.synchronize()
        done += 8
        dt = time.perf_counter() - t0
        if (stop is not None and stop()) or (stop is None and dt >= seconds):
            return 2.0 * n ** 3 * done / dt / 1e12, dt


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 32.0
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    codec = sys.argv[4] if len(sys.argv) > 4 else "tpz1"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    state = synthetic_checkpoint(int(gb * 1e9), 8192, dev)
    a = torch.randn(n, n, dtype=torch.bfloat16, device=dev)
    b = torch.randn(n, n, dtype=torch.bfloat16, device=dev)
    ck = Checkpointer(state, codec=codec, chunk_bytes=chunk << 20)
    ck.save_async({"warm": True}).result()  # snapshot buffer, engine and codec buffers
    gemm_rate(a, b, 1.0)  # warm the GEMM
    alone, _ = gemm_rate(a, b, 3.0)
    t = time.perf_counter()
    ck.save_async({"step": 1}).result()
    spill_alone = time.perf_counter() - t
    pending = ck.save_async({"step": 2})
    t = time.perf_counter()
    shared, dt = gemm_rate(a, b, 0.0, stop=pending.done)
    pending.result()
    spill_shared = time.perf_counter() - t
    out = {"state_GB": round(ck.plan.total / 1e9, 1), "gemm_n": n, "chunk_MiB": chunk,
           "codec": codec,
           # GEMM work the spill cost: the window's shortfall against the loop alone
           "gemm_seconds_lost": round(dt * (1 - shared / alone), 3),
           "gemm_TFLOPs_alone": round(alone, 1), "gemm_TFLOPs_during_spill": round(shared, 1),
           "gemm_slowdown": round(1 - shared / alone, 3), "gemm_window_s": round(dt, 3),
           "spill_s_alone": round(spill_alone, 3), "spill_s_with_gemm": round(spill_shared, 3),
           "stall_ms": round(pending.stall_s * 1e3, 2)}
    print(out, flush=True)
    ck.close()


if __name__ == "__main__":
    main()
