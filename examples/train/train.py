#!/usr/bin/env python3
"""Example rank workload for ``iterative_task`` on ``cloud = "mi355x"``.

* stages the task workdir into HBM (rank 0 reads, RCCL fans out to the other ranks),
* trains a small random-init transformer-style MLP in bf16 on synthetic tokens (DDP over
  RCCL when ``WORLD_SIZE > 1``),
* checkpoints model + optimizer state to host DRAM on SIGTERM (preemption) at the next step
  boundary (``state.step``) -- all ranks at the same step -- and resumes from it when
  respawned, persisting to the task's storage at the end.

Environment (set by the supervisor): RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT,
HIP_VISIBLE_DEVICES, TPI_DATA_DIRECTORY, TPI_MACHINE_IDENTITY.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.environ.get("TPI_FRAMEWORK_ROOT") or os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def log(*parts):
    print(*parts, flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--hidden", type=int, default=2048)
    p.add_argument("--layers", type=int, default=4)
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--seq", type=int, default=512)
    p.add_argument("--stage", action="store_true", help="stage the workdir into HBM first")
    p.add_argument("--sleep", type=float, default=0.0, help="sleep per step (tests)")
    p.add_argument("--ckpt-every", type=int, default=0,
                   help="asynchronous checkpoint every N steps (0: only on SIGTERM/exit)")
    p.add_argument("--materialize", action="store_true",
                   help="resume by materializing the state from the spill (the model is built "
                        "on the meta device; for ranks bigger than half of HBM; one rank)")
    args = p.parse_args()
    # first log line before the framework import (~0.5-1.5 s): the task is visibly running
    # while torch loads and the runtime stages the workdir (attach() waits for it below)
    log("rank %s/%s starting (machine %s)" % (os.environ.get("RANK", "0"),
                                             os.environ.get("WORLD_SIZE", "1"),
                                             os.environ.get("TPI_MACHINE_IDENTITY", "-")))

    import torch
    import torch.distributed as dist

    from terraform_provider_iterative_amd.checkpoint import TrainingState, preemption

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    data_dir = os.environ.get("TPI_DATA_DIRECTORY", ".")
    spill = os.path.join(data_dir, ".ckpt-rank%d" % rank)
    # warm standby: a successor started while its preempted predecessor is still spilling waits
    # here (torch imported, GPU up, spill region being mapped) until the supervisor activates it
    materialize = args.materialize and device.type == "cuda" and world == 1
    preemption.standby(spill if device.type == "cuda" else None, materialize=materialize)
    if world > 1:
        dist.init_process_group("nccl" if device.type == "cuda" else "gloo",
                                **({"device_id": device} if device.type == "cuda" else {}))
    log("rank %d/%d on %s (machine %s)" % (rank, world, device,
                                          os.environ.get("TPI_MACHINE_IDENTITY", "-")))
    stats = {}
    if args.stage and os.environ.get("TPI_HBM_WORKDIR"):
        # the runtime staged the workdir before this rank started (tpi-stager): map it
        from terraform_provider_iterative_amd.runtime.stage import attach

        t0 = time.perf_counter()
        staged = attach()
        stats["attach_s"] = time.perf_counter() - t0
        stats["stage_GBps"] = staged.stats.get("staged_GBps")
        stats.update({k: v for k, v in staged.stats.items() if isinstance(v, (int, float, bool, str))})
        log("workdir in HBM: %d files, %.2f GB, attached in %.4fs (%s)" % (
            len(staged.files), staged.total / 1e9, stats["attach_s"], json.dumps(stats)))
    elif args.stage:  # staging disabled for the task (TPI_STAGE=off / small): do it here
        from terraform_provider_iterative_amd.runtime.workdir import stage_workdir

        t0 = time.perf_counter()
        staged = stage_workdir(device=device, exclude=[".ckpt*", "checkpoints"])
        dt = time.perf_counter() - t0
        stats["stage_GBps"] = staged.stats["bytes"] / dt / 1e9 if dt else None
        stats.update({k: v for k, v in staged.stats.items() if isinstance(v, (int, float, bool, str))})
        log("staged %d files, %.2f GB into HBM in %.3fs (%s)" % (
            len(staged.files), staged.stats["bytes"] / 1e9, dt, json.dumps(stats)))

    torch.manual_seed(1234)
    h = args.hidden

    def build():
        layers = []
        for _ in range(args.layers):
            layers += [torch.nn.LayerNorm(h), torch.nn.Linear(h, 4 * h), torch.nn.GELU(),
                       torch.nn.Linear(4 * h, h)]
        return torch.nn.Sequential(*layers)

    def make_opt(m):
        return torch.optim.AdamW(m.parameters(), lr=1e-4)

    # the batch generator: part of the checkpoint, so a resumed run draws the batches the
    # uninterrupted one would have (not the first batches again)
    gen = torch.Generator(device=device).manual_seed(rank + 7)
    got = preemption.materialize(spill, device) if materialize else None
    if got is not None:
        # the state is created while it streams in from the predecessor: no up-front
        # allocation of a model that would not fit next to the predecessor's
        with torch.device("meta"):
            model = build().to(torch.bfloat16)
        state = TrainingState.from_materialized(got, model, make_opt, generators={"data": gen})
        opt, step_t, meta = state.optimizer, got[1]["extra.step"], got[2]
    else:
        model = build().to(device=device, dtype=torch.bfloat16)
        opt = make_opt(model)
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model)
        step_t = torch.zeros((), dtype=torch.int64, device=device)
        # Optimizer state must exist before it can be checkpointed: one warm step on zeros.
        x = torch.zeros(args.batch, args.seq, h, device=device, dtype=torch.bfloat16)
        model(x).float().pow(2).mean().backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        # model + optimizer device state by reference; CPU-side Adam step counters, the
        # optimizer hyper-parameters, every RNG and `gen` ride in the checkpoint header
        state = TrainingState(model, opt, extra={"step": step_t}, path=spill,
                              generators={"data": gen})
        # ranks agree on the step to resume from (or all start fresh)
        meta = state.resume_consistent() if world > 1 else state.resume()
    ck = state.checkpointer
    start = int(step_t.item())
    log("resumed from step %d" % start if meta else "fresh start")
    state.install()

    t_steps, stalls = [], []
    for step in range(start, args.steps):
        t0 = time.perf_counter()
        x = torch.randn(args.batch, args.seq, h, device=device, dtype=torch.bfloat16,
                        generator=gen)
        loss = (model(x).float() - x.float()).pow(2).mean()
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        step_t.fill_(step + 1)
        if device.type == "cuda":
            torch.cuda.synchronize()
        t_steps.append(time.perf_counter() - t0)
        if rank == 0 and (step % 10 == 0 or step + 1 == args.steps):
            log("step %d loss %.5f" % (step + 1, loss.item()))
        if args.sleep:
            time.sleep(args.sleep)
        t_ck = time.perf_counter()
        if args.ckpt_every and (step + 1) % args.ckpt_every == 0:
            state.save_async({"step": step + 1})  # HBM snapshot; the PCIe spill runs behind
        # step boundary: a SIGTERM that arrived during this step is saved here (every rank at
        # the same step); periodic checkpoints every TPI_SYNC_INTERVAL s (default 10)
        elif not state.step(step + 1):
            continue
        if device.type == "cuda":
            torch.cuda.current_stream().synchronize()
        stalls.append(time.perf_counter() - t_ck)
    res = state.save({"step": int(step_t.item()), "final": True})
    if stalls:
        stats["ckpt_stall_ms"] = 1e3 * max(stalls)
    if t_steps:
        stats["step_ms"] = 1e3 * sorted(t_steps)[len(t_steps) // 2]
    stats["final_save_GBps"] = res.gbps
    log("done %s" % json.dumps(stats))
    ck.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
