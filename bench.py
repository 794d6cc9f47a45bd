#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): checkpoint save/restore GB/s + apply->first-log latency.

Config "Preempt-recover: 100 GB checkpoint pack -> host DRAM -> restore": the 100 GB
checkpoint (bf16 parameters + fp32 Adam moments of a synthetic transformer, random init) is
sharded over the N ranks (one per GPU, ``torch.distributed`` over RCCL when N > 1), so the
total work is fixed: strong scaling.  One step = save (pack + CRC32C tiles [+ TPZ1 byte-plane
encode] -> pinned host DRAM over PCIe, side-stream pipeline) + restore (host -> HBM [decode],
verify every tile's CRC32C, scatter).  The codec is lossless; ``value`` counts checkpoint
(tensor) bytes, the JSON also reports the compressed bytes that crossed PCIe.

The restore is the one a preempted rank's successor runs (config 4's streamed hand-off, the
runtime default): it restores the checkpoint *being* saved into the successor's own tensors,
chunk by chunk as the save publishes them, over the other direction of the PCIe link.  Both
are complete and verified inside every step; ``--no-overlap`` restores only after the save
(into the saved tensors), and the JSON also carries that sequential rate (``sequential``).

Synthetic state (random, no dataset/checkpoint available): bf16 parameters ~ N(0, 0.02),
fp32 exp_avg ~ N(0, 1e-3), fp32 exp_avg_sq ~ N(0, 1e-3)^2 -- value distributions of a
trained AdamW state (an untrained one would be all-zero moments, which compress ~1000x).

    python bench.py --gpus N --steps K --warmup W

Rank 0 prints one JSON line.  ``value`` = checkpoint bytes moved (save + restore, both
directions counted together: they run at once on the two directions of the PCIe link) by all
ranks per second of wall time (max over ranks of the timed region).  Untimed side
measurements, none of them part of ``value``:

* before the timed region: task apply -> first-log latency of an ``iterative_task`` on the
  node-local runtime (``first_log_latency_s``), and on one GPU BASELINE config 2 -- ``tpi
  apply`` of a 10 GB workdir + ``train.py`` on an idle GPU (``first_log_latency_config2``:
  first log, push, staging);
* after it: async-save stall, raw (codec-free) rates, the workdir fan-out, the sequential
  rate, and on one GPU config 4 end to end through the product (``preempt_e2e``: cold =
  the default preloaded successor, hot standby, fresh process; each run's own memory gates --
  ``gpu_drain``, ``successor_hbm_wait`` -- are reported, the bench adds no wait of its own).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("task apply→first-log latency (s) + checkpoint save/restore GB/s, "
          "1/2/4/8 GPU")
CONFIG_NAME = ("Preempt-recover: SIGTERM mid-task, 100 GB checkpoint pack→host "
               "DRAM→restore")


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--total-gb", type=float, default=100.0,
                   help="checkpoint size summed over all ranks (GB, 1e9 bytes)")
    p.add_argument("--mode", choices=("sdma", "direct"), default="sdma",
                   help="sdma: staged pipeline, D2H on an SDMA copy engine (d2h_engine in the "
                        "JSON; TPI_D2H_ENGINE=blit for HIP's blit kernels), H2D on HIP's copy "
                        "engine; direct: kernels read/write host-mapped memory")
    p.add_argument("--codec", choices=("none", "tpz1"), default="tpz1")
    p.add_argument("--tile-mb", type=float, default=1.0)
    p.add_argument("--chunk-mb", type=float, default=256.0)
    p.add_argument("--nbuf", type=int, default=4,
                   help="staging buffers per engine (4: +0.8 %% over 3 in alternating runs, "
                        "profiles/pipeline_depth_round3.md)")
    p.add_argument("--hidden", type=int, default=8192)
    p.add_argument("--no-latency", action="store_true", help="skip apply->first-log")
    p.add_argument("--broadcast-gb", type=float, default=10.0,
                   help="also measure staging a workdir of this many GB into HBM on every "
                        "rank (N>1: sharded H2D + xGMI all-gather vs RCCL broadcast vs "
                        "independent H2D)")
    p.add_argument("--verify", action="store_true", default=True)
    p.add_argument("--no-async", action="store_true",
                   help="skip the (untimed) save_async stall measurement")
    p.add_argument("--side-timeout", type=float, default=300.0,
                   help="seconds the untimed side measurements may take before rank 0 prints "
                        "the headline without them")
    p.add_argument("--no-overlap", action="store_true",
                   help="restore after the save instead of streaming behind it")
    p.add_argument("--spill-dir", default="/dev/shm",
                   help="where the host region lives (shared by saver and restorer)")
    p.add_argument("--strict-numa", action="store_true",
                   help="stop before the timed steps (exit 4) when a rank's host region is not "
                        "on its GPU's socket (default: warn, measure, and name the ranks in "
                        "rank_placement.remote_numa_ranks)")
    p.add_argument("--preempt-e2e", choices=("auto", "none"), default="auto",
                   help="auto (1 GPU): after everything else, untimed, preempt a real "
                        "iterative_task holding --total-gb of state twice (cold successor, hot "
                        "standby) and report signal -> restored (preempt_e2e)")
    p.add_argument("--config2", choices=("auto", "none"), default="auto",
                   help="untimed, 1 GPU: apply -> first log of BASELINE config 2 (10 GB "
                        "workdir + train.py) through tpi apply (first_log_latency_config2)")
    p.add_argument("--e2e-timeout", type=float, default=420.0,
                   help="seconds each preempt_e2e run may take")
    p.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                   help="cpu: rehearse the multi-rank control flow on CPU tensors over gloo "
                        "(tests; not a measurement of the MI355X path)")
    return p.parse_args(argv)


def synthetic_checkpoint(nbytes: int, hidden: int, device, fill: bool = True):
    """bf16 weights + fp32 AdamW moments of transformer blocks until ``nbytes`` is reached
    (``fill=False``: uninitialised, for a process that is about to restore them)."""
    import torch

    h = hidden
    ffn = int(8 * h / 3 + 255) // 256 * 256
    block = [("attn.qkv", (3 * h, h)), ("attn.out", (h, h)), ("mlp.up", (2 * ffn, h)),
             ("mlp.down", (h, ffn)), ("norm1", (h,)), ("norm2", (h,))]
    tensors, used, layer = {}, 0, 0
    gen = torch.Generator(device=device).manual_seed(1234)
    while used < nbytes:
        for name, shape in block:
            numel = 1
            for s in shape:
                numel *= s
            for kind, dtype in (("param", torch.bfloat16), ("exp_avg", torch.float32),
                                ("exp_avg_sq", torch.float32)):
                esz = torch.empty((), dtype=dtype).element_size()
                left = nbytes - used
                if left <= 0:
                    break
                n = min(numel, max(left // esz, 1))
                t = torch.empty(n if n != numel else shape, dtype=dtype, device=device)
                if not fill:
                    pass
                elif kind == "param":
                    t.normal_(0, 0.02, generator=gen)
                elif kind == "exp_avg":
                    t.normal_(0, 1e-3, generator=gen)
                else:
                    t.normal_(0, 1e-3, generator=gen)
                    t.mul_(t)
                tensors["layers.%d.%s.%s" % (layer, name, kind)] = t
                used += t.numel() * esz
        layer += 1
    return tensors


def first_log_latency(timeout: float = 60.0, parallelism: int = 1):
    try:
        from terraform_provider_iterative_amd.bench_latency import measure_first_log_latency
    except ImportError:
        return None
    try:
        return measure_first_log_latency(timeout=timeout, parallelism=parallelism)
    except Exception as error:  # the headline must not die on the latency probe
        print("bench: first-log latency probe failed: %s" % error, file=sys.stderr)
        return None


E2E_KEYS = ("ok", "verified", "status", "signal_to_restored_s", "save_s",
            "rank_start_to_restored_s", "saved_to_restored_s", "signal_to_durable_s", "streamed",
            "warm_standby_activated", "hot_standby", "preload", "preloaded_wait_s", "preload_gpu",
            "standby_pinned_wait_s", "restore_journal",
            "extra_tensors_gib", "delete_s", "rank_exit_to_settled_s", "gpu_drain",
            "successor_hbm_wait", "hbm_failed", "hbm_fault_dumps", "hbm_skipped",
            "timeline_on_failure",
            "memory_guard",
            "released_exit_pending_at_settle")


def preempt_e2e(total_gb: float, codec: str, timeout: float) -> dict:
    """Config 4's real path, untimed: an ``iterative_task`` on ``cloud = "mi355x"`` holding
    ``total_gb`` of state in HBM is preempted (``leo preempt``: SIGTERM to the rank), the
    supervisor respawns it and the successor restores and verifies the state
    (``bench/bench_preempt.py``, one child process per run).  ``cold``: no standby -- the
    successor the default configuration gives (a preloaded interpreter, runtime/preload.py,
    that imported PyTorch before the preemption); ``fresh``: ``TPI_PRELOAD=0``, a new process;
    ``hot``: a hot standby started with the rank copies the state device to device.  Signal ->
    restored is read from the task's phase journal."""
    import subprocess

    runs = {}
    # the hot run's state also holds a 4.2 GiB and a 2.5 GiB tensor (a large vocabulary's fp32
    # embedding and moments): allocations HIP IPC cannot hand off, the dma-buf route can
    for name, flags in (("cold", []), ("hot", ["--hot", "--extra-gib", "4.2,2.5"]),
                        ("fresh", ["--no-preload"])):
        cmd = [sys.executable, os.path.join(ROOT, "bench", "bench_preempt.py"), "--gb",
               repr(total_gb), "--codec", codec, "--timeout", repr(timeout)] + flags
        t0 = time.perf_counter()
        try:
            proc = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout + 120)
            lines = [l for l in proc.stdout.splitlines() if l.startswith("{")]
            if proc.returncode != 0 or not lines:
                runs[name] = {"error": "exit %d: %s" % (proc.returncode, proc.stderr[-600:])}
                continue
            result = json.loads(lines[-1])
        except Exception as error:  # never lose the headline to the side measurement
            runs[name] = {"error": repr(error)}
            continue
        runs[name] = {k: result.get(k) for k in E2E_KEYS}
        runs[name]["wall_s"] = round(time.perf_counter() - t0, 1)
        print("bench: preempt_e2e %s: signal -> restored %s s, verified %s" % (
            name, result.get("signal_to_restored_s"), result.get("verified")),
            file=sys.stderr, flush=True)
    return {"cold_signal_to_restored_s": runs.get("cold", {}).get("signal_to_restored_s"),
            "hot_signal_to_restored_s": runs.get("hot", {}).get("signal_to_restored_s"),
            "fresh_signal_to_restored_s": runs.get("fresh", {}).get("signal_to_restored_s"),
            "verified": all(r.get("ok") is True for r in runs.values()),
            "gb": total_gb, "runs": runs}


def workdir_config2(gb: float, timeout: float) -> dict:
    """BASELINE config 2 through the product, untimed: ``tpi apply`` of a
    ``gb`` GB synthetic workdir + PyTorch-ROCm ``examples/train/train.py`` on ``mi355x``
    (``bench/bench_workdir.py``, one child process).  ``first_log_s``: apply -> the task's
    first log line; ``push_s`` / ``push_method``: the workdir's push into task storage as the
    task journalled it (reflinked where the filesystem can, else copied); ``stage_s``: rank
    start -> the stager's HBM image published (it runs beside the rank's start-up)."""
    import subprocess

    cmd = [sys.executable, os.path.join(ROOT, "bench", "bench_workdir.py"), "--gb", repr(gb),
           "--steps", "2", "--files", "10"]
    t0 = time.perf_counter()
    try:
        proc = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
        lines = [l for l in proc.stdout.splitlines() if l.startswith("{")]
        if proc.returncode != 0 or not lines:
            return {"error": "exit %d: %s" % (proc.returncode, proc.stderr[-600:])}
        r = json.loads(lines[-1])
    except Exception as error:  # never lose the headline to the side measurement
        return {"error": repr(error)}
    out = {"first_log_s": r.get("apply_to_first_log_s"), "push_s": r.get("push_s"),
           "push_method": r.get("push_method"), "stage_s": r.get("stage_s"),
           "gpu_drain": r.get("gpu_drain"),
           "apply_s": r.get("apply_s"), "stage_GBps": r.get("stage_GBps"),
           "train_step_ms": r.get("train_step_ms"), "workdir_gb": gb,
           "ok": bool(r.get("apply_ok") and r.get("stage_GBps")),
           "wall_s": round(time.perf_counter() - t0, 1)}
    print("bench: config2 apply -> first log %s s (push %s s, %s; stage %s s)" % (
        out["first_log_s"], out["push_s"], out["push_method"], out["stage_s"]),
        file=sys.stderr, flush=True)
    return out


def launch_ranks(args, argv) -> int:
    """``--gpus N`` without a launcher around us: start the N ranks ourselves (one process
    per GPU, the same env contract as ``torch.distributed.run``), before anything here touches
    the GPU, and exit with the first failing rank's code.  Only rank 0 prints the JSON line."""
    import signal
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    argv = list(sys.argv[1:] if argv is None else argv)
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print("bench: rank %d exited with %d; stopping the others"
                          % (procs.index(p), code), file=sys.stderr)
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        rc = 130
    return rc


def host_memory_check(per_rank: int, local_world: int) -> None:
    """Each rank keeps its checkpoint region in (NUMA-local, pinned) host DRAM: refuse to
    start when the node cannot hold all of them rather than letting the OOM killer pick."""
    try:
        with open("/proc/meminfo") as f:
            info = {l.split(":")[0]: int(l.split()[1]) * 1024 for l in f if ":" in l}
    except (OSError, ValueError, IndexError):
        return
    avail = info.get("MemAvailable")
    need = int(per_rank * 1.02) * local_world  # region = stream + headers + codec bound
    if avail is not None and need > avail:
        raise SystemExit("bench: %d ranks x %.1f GB host regions need %.1f GB, only %.1f GB "
                         "available" % (local_world, per_rank / 1e9, need / 1e9, avail / 1e9))


def main(argv=None):
    args = parse_args(argv)
    # HIP spreads a process's streams over GPU_MAX_HW_QUEUES hardware queues (4 by default).
    # The saving and the restoring engine hold 8 streams between them; on 4 queues the save's
    # kernels can sit behind the restore's cross-stream waits, idling the save's PCIe leg
    # (117-119 -> 121 GB/s with 8 queues, profiles/hw_queues_round3.md).  Set before the
    # first HIP call, inherited by ranks this process launches.
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args, argv))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench: WORLD_SIZE=%d but --gpus=%d: the launcher and the flags "
                         "disagree" % (world, args.gpus))
    on_gpu = args.device == "cuda"
    if on_gpu and not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (MI355X)")
    # TPI_BENCH_BACKEND=gloo rehearses the multi-rank flow on a box with fewer GPUs than ranks
    # (ranks then share devices); the real runs use RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("TPI_BENCH_BACKEND", "nccl") if on_gpu else "gloo"
    pinned_cpus = None
    if on_gpu:
        ndev = torch.cuda.device_count()
        if backend == "nccl" and world > ndev:
            raise SystemExit("bench: %d ranks but %d visible GPUs (RCCL needs one GPU per rank)"
                             % (world, ndev))
        index = local_rank % ndev
        torch.cuda.set_device(index)
        device = torch.device("cuda", index)
        # host side of the rank (pinned region first touch, CRC combine, codec bookkeeping)
        # on the cores of the GPU's own socket
        from terraform_provider_iterative_amd.parallel.placement import pin_to_device_numa

        pinned_cpus = pin_to_device_numa(index)
    else:
        device = torch.device("cpu")
    host_memory_check(int(args.total_gb * 1e9 / world),
                      int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    rccl_dir = None
    if world > 1 and backend == "nccl":
        # RCCL's own account of the communicator (rank count, transport per peer link),
        # parsed after the timed loop: evidence that N ranks met over xGMI (P2P), not SHM
        import tempfile

        from terraform_provider_iterative_amd.parallel import rccl_log

        rccl_dir = os.path.join(tempfile.gettempdir(), "tpi-bench-rccl-%s" % os.environ.get(
            "MASTER_PORT", "0"))
        os.environ.update(rccl_log.debug_env(rccl_dir))
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()
        sync()

    def allmax(value: float) -> float:
        if world == 1:
            return value
        t = torch.tensor([value], dtype=torch.float64,
                         device=device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    latency = None
    if rank == 0 and not args.no_latency:
        # an iterative_task with parallelism = N (one GPU per rank), like the job measured
        # (one GPU per rank: a rehearsal with more ranks than GPUs probes with what exists).
        # Measured first: a process that already maps the 100 GB host region and the HBM
        # state spawns the probe's `tpi apply` ~17 ms slower (profiles/hw_queues_round3.md).
        gpus = torch.cuda.device_count() if on_gpu else world
        latency = first_log_latency(parallelism=max(1, min(world, gpus)))
        if latency:
            print("bench: apply -> first log %s s (CLI), %s s (API); GPU memory gate waited "
                  "up to %s s" % (latency.get("cli_s"), latency.get("api_s"),
                                  latency.get("gpu_drain_max_s")), file=sys.stderr, flush=True)
    config2 = None
    if rank == 0 and world == 1 and on_gpu and args.config2 == "auto":
        # config 2 as a user meets it: on an idle GPU, before this process fills the device
        # (after the timed loop the driver is still taking back its 200 GB, and the task's
        # start would rightly wait for that: gpu-drain)
        config2 = workdir_config2(10.0, args.e2e_timeout)
    if world > 1:
        # the other ranks start their setup (filling and pinning their share of the state)
        # only after rank 0's probes: N-1 setups beside it inflated the measured first log
        # (rehearsal with 4 ranks on one GPU: 0.217 s against 0.073 s, profiles/round6/r6j)
        barrier()

    from terraform_provider_iterative_amd.checkpoint import Checkpointer

    per_rank = int(args.total_gb * 1e9 / world)
    overlap = not args.no_overlap
    spill_dir = args.spill_dir if os.path.isdir(args.spill_dir) else None
    import tempfile

    spill_path = os.path.join(spill_dir or tempfile.gettempdir(), "tpi-bench-%s-%d-r%d.spill" % (
        os.environ.get("MASTER_PORT", "0"), os.getpid(), rank))
    t_setup = time.perf_counter()
    tensors = synthetic_checkpoint(per_rank, args.hidden, device)
    sync()
    ck_kw = dict(tile_bytes=int(args.tile_mb * (1 << 20)), chunk_bytes=int(args.chunk_mb * (1 << 20)),
                 nbuf=args.nbuf, mode=args.mode, codec=args.codec)
    ck = Checkpointer(tensors, path=spill_path, **ck_kw)
    successor = ck_in = None
    if overlap:  # the successor's tensors, restored from the same host region
        successor = synthetic_checkpoint(per_rank, args.hidden, device, fill=False)
        sync()
        ck_in = Checkpointer(successor, path=spill_path, **ck_kw)
    try:  # both mappings hold the pages; no name left behind even if the process dies
        os.remove(spill_path)
    except OSError:
        pass
    setup_s = time.perf_counter() - t_setup

    barrier()

    def save_restore(meta):
        """One step: (wire bytes, save s, restore s, restore result)."""
        a = time.perf_counter()
        if not overlap:
            wire = ck.save(meta).wire_bytes
            b = time.perf_counter()
            res = ck.restore()
            return wire, b - a, time.perf_counter() - b, res
        box = {}

        def restorer():
            try:
                box["res"] = ck_in.restore()
            except BaseException as error:  # surfaced below
                box["error"] = error
            box["t"] = time.perf_counter()

        thread = threading.Thread(target=restorer, name="bench-restore")
        # the restore starts once the save has published its streaming header
        wire = ck.save(meta, on_stream=thread.start).wire_bytes
        b = time.perf_counter()
        thread.join()
        if "error" in box:
            raise box["error"]
        return wire, b - a, box["t"] - a, box["res"]

    def progress(msg: str) -> None:  # stderr heartbeat: long (profiled) runs are not silent
        if rank == 0:
            print("bench: " + msg, file=sys.stderr, flush=True)

    progress("setup %.1f s (%d bytes per rank)" % (setup_s, per_rank))
    for i in range(args.warmup):
        save_restore({"warmup": True})
        progress("warmup %d/%d" % (i + 1, args.warmup))
    # Where each rank's host region landed vs its GPU's socket, gathered from every rank: at
    # N = 8 the overlapped step moves ~0.74 TB/s through host DRAM over two sockets, and a
    # region on the wrong socket also crosses the inter-socket link.  Checked after the warmup
    # (its saves touched every page of the regions), before timing.
    from terraform_provider_iterative_amd.checkpoint.host import numa_placement
    from terraform_provider_iterative_amd.parallel.placement import region_placement_report

    gpu_numa = -1
    if on_gpu:
        import ctypes

        from terraform_provider_iterative_amd.ops import hip

        node = ctypes.c_int(-1)
        if hip().tpi_device_numa_node(device.index, ctypes.byref(node)) == 0:
            gpu_numa = node.value
    elif os.environ.get("TPI_FAKE_GPU_NUMA"):  # CPU rehearsal of a multi-socket node
        fake = [int(v) for v in os.environ["TPI_FAKE_GPU_NUMA"].split(",")]
        gpu_numa = fake[local_rank % len(fake)]
    placed = numa_placement(ck.region.addr, ck.region.size) if ck.region is not None else None
    mine = {"rank": rank, "gpu_numa": gpu_numa,
            "bytes_per_node": (placed or {}).get("bytes_per_node", {}),
            "policy": (placed or {}).get("policy"),
            "cpus": len(pinned_cpus) if pinned_cpus else None}

    def gather(obj):
        if world == 1:
            return [obj]
        objs = [None] * world
        dist.all_gather_object(objs, obj)
        return objs

    placements = gather(mine)
    # every rank's view of the job's communicators (gathered; RCCL fields null under gloo)
    comm_mine = {"rank": rank, "backend": backend if world > 1 else None,
                 "torch_pg_size": dist.get_world_size() if world > 1 else 1, "rccl": None}
    if rccl_dir is not None:
        from terraform_provider_iterative_amd.parallel import rccl_log

        comm_mine["rccl"] = rccl_log.parse_files(os.path.join(rccl_dir, "rccl-%d.log" % os.getpid()))
    comm_ranks = gather(comm_mine)
    _, numa_problems = region_placement_report(placements)
    if numa_problems:
        if rank == 0:
            print("bench: WARNING: host regions off their GPU's socket (their copies also "
                  "cross the inter-socket link): " + "; ".join(numa_problems), file=sys.stderr,
                  flush=True)
        if args.strict_numa:
            raise SystemExit(4)
    barrier()

    fault = os.environ.get("TPI_BENCH_FAULT", "")
    if fault and fault != "skip-restore-after-first":
        raise SystemExit("bench: unknown TPI_BENCH_FAULT %r" % fault)

    def poison(tensors_):
        """Overwrite every successor tensor with a pattern no checkpoint holds (outside the
        timed window): only a restore that rewrites all of them passes the final digest check."""
        for t in tensors_.values():
            t.view(-1).view(torch.uint8).fill_(0xA5)

    if fault:  # fault injection for the contract test: a restore that stops rewriting
        real_restore = ck_in.restore if ck_in is not None else ck.restore
        calls = [0]

        def broken_restore(*a, **kw):
            res = real_restore(*a, **kw)
            calls[0] += 1
            if calls[0] > 1:  # "skips" tensors 3.. after the first timed step
                poison(dict(list((successor or tensors).items())[2:]))
            return res

        if ck_in is not None:
            ck_in.restore = broken_restore
        else:
            ck.restore = broken_restore

    save_s = restore_s = 0.0
    wire = split_chunks = 0
    elapsed = 0.0
    for step in range(args.steps):
        if overlap and successor is not None:
            poison(successor)  # untimed: the restore must rewrite every successor tensor
        barrier()
        t0 = time.perf_counter()
        wire, s_s, r_s, res = save_restore({"step": step})
        barrier()
        elapsed += time.perf_counter() - t0
        if ck_in is not None and ck_in.engine is not None:  # duplex balancing of this step
            split_chunks += ck_in.engine.split_chunks
        if res.bad_tiles:
            raise SystemExit("bench: %d corrupt tiles after restore" % res.bad_tiles)
        save_s += s_s
        restore_s += r_s
        progress("step %d/%d save %.3f s restore %.3f s" % (step + 1, args.steps, s_s, r_s))

    verified = None
    if args.verify:  # outside the timed region: prove the restore really rewrote HBM
        from terraform_provider_iterative_amd import ops

        def digest(d, n):
            out = ops.shard_hash(d[n].view(-1).view(torch.uint8))
            return out.cpu().tolist() if hasattr(out, "cpu") else out.tolist()

        if overlap:  # every tensor of the successor (poisoned before the last step) equals
            sync()   # the saved state
            verified = all(digest(successor, n) == digest(tensors, n) for n in tensors)
        else:
            names = list(tensors)[:3]
            before = [digest(tensors, n) for n in names]
            for n in names:
                tensors[n].zero_()
            ck.restore()
            sync()
            verified = before == [digest(tensors, n) for n in names]
        if world > 1:  # the job is verified only if every rank's restore is
            verified = verified and allmax(0.0 if verified else 1.0) == 0.0
    if ck_in is not None:  # the side measurements need the HBM back
        ck_in.close()
        ck_in = None
        successor = None
        if on_gpu:
            torch.cuda.empty_cache()

    host_numa = placed if rank == 0 else None  # rank 0's spill pages (kept for history)
    # every rank's region moves its wire bytes into host DRAM (save) and out again (restore)
    wires = gather(int(wire))
    for entry, w in zip(placements, wires):
        entry["wire_bytes_per_step"] = 2 * w
    placement_report, _ = region_placement_report(placements)
    placement_report["remote_numa_ranks"] = numa_problems
    elapsed = allmax(elapsed)
    save_max, restore_max = allmax(save_s), allmax(restore_s)

    total = ck.plan.total * world  # packed bytes per direction per step (all ranks)
    wire_total = int(allmax(float(wire))) * world  # (upper bound: max rank x N)
    value = 2 * total * args.steps / elapsed / 1e9
    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": ("synthetic random AdamW state: bf16 params N(0,0.02), fp32 exp_avg "
                     "N(0,1e-3), fp32 exp_avg_sq N(0,1e-3)^2"
                     + ("" if on_gpu else "; CPU rehearsal, not an MI355X measurement")),
            "config": {"model": CONFIG_NAME, "global_batch": 1, "seq_len": None,
                       "parallelism": "shard%d" % world, "checkpoint_bytes": total,
                       "tile_bytes": ck.plan.tile_bytes,
                       "chunk_bytes": ck.engine.chunk_bytes if ck.engine else None,
                       "mode": args.mode, "codec": args.codec,
                       "d2h_engine": ck.engine.d2h_engine if ck.engine else None,
                       "tensors_per_rank": len(tensors),
                       # HIP hardware queues per process, as run: the MI355X boxes export 4
                       # (HIP's default, the runtime ranks' too); bench.py asks for 8 only
                       # where nothing is set (+2-3 %%, profiles/hw_queues_round3.md)
                       "gpu_max_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       # every runtime knob set in the environment, by name
                       "env_knobs": {k: v for k, v in sorted(os.environ.items())
                                     if k.startswith(("TPI_", "GPU_", "HSA_", "HIP_", "AMD_",
                                                      "PYTORCH_HIP", "NCCL_", "RCCL_"))}},
            # what the timed loop is: one process saves the state (pack + CRC32C tiles +
            # TPZ1 -> pinned host DRAM) while a successor Checkpointer restores it behind the
            # save; the SIGTERM -> respawn -> restore of a real iterative_task is measured
            # after it, untimed, in preempt_e2e
            "timed_loop": "in-process save streamed to a successor restore (both verified)",
            "preempt_e2e": None,
            # per rank: torch process-group size, backend, RCCL's rank count and transports
            "comm": {"ranks": comm_ranks,
                     "pg_sizes_match": all(c["torch_pg_size"] == world for c in comm_ranks),
                     "rccl_nranks_match": (all((c["rccl"] or {}).get("nranks") == world
                                               for c in comm_ranks) if rccl_dir else None),
                     "rccl_xgmi_only": (all((c["rccl"] or {}).get("xgmi_only") is True
                                            for c in comm_ranks) if rccl_dir else None)},
            # what `value` counts: checkpoint bytes saved + restored per second, the restore
            # streaming behind the save over the other direction of the PCIe link (the
            # preemption hand-off's streamed route); rounds 1-2 measured save-then-restore,
            # which is `value_sequential` below
            "value_kind": "overlapped_duplex" if overlap else "sequential",
            "value_sequential": None,
            "save_GBps": round(total * args.steps / save_max / 1e9, 3),
            "restore_GBps": round(total * args.steps / restore_max / 1e9, 3),
            "restore_streams_behind_save": overlap,
            # chunks of the timed restores whose H2D went over two copy streams: the safety
            # valve for a restore trailing the save by TPI_H2D_SPLIT_LEAD chunks.  0 is the
            # healthy value -- the bounded run-ahead keeps the restore within a chunk of the
            # save (profiles/duplex_split_round3.md section 4)
            "restore_split_chunks": split_chunks if overlap else None,
            "per_gpu_save_GBps": round(ck.plan.total * args.steps / save_max / 1e9, 3),
            "per_gpu_restore_GBps": round(ck.plan.total * args.steps / restore_max / 1e9, 3),
            "wire_bytes_per_step": wire_total,
            "compression_ratio": round(wire_total / total, 4),
            "save_wire_GBps": round(wire_total * args.steps / save_max / 1e9, 3),
            "first_log_latency_s": (latency or {}).get("cli_s"),
            "first_log_latency": latency,
            "workdir_broadcast": None,
            "raw_GBps": None,
            "sequential": None,
            "rank0_cpu_affinity": len(pinned_cpus) if pinned_cpus else None,
            "host_region_numa": host_numa,
            # per rank: GPU socket, where its host region's pages are, the bytes it moves
            # through host DRAM per step; and the per-socket totals
            "rank_placement": placement_report,
            "restore_verified": verified,
            "save_async": None,
            "setup_s": round(setup_s, 2),
        }

    # Side measurements (collectives) run under a watchdog: should one of them hang, rank 0
    # still prints the headline line, marked, and every rank leaves without the hung call.
    printed = threading.Lock()

    def emit(note=None):
        if out is not None and printed.acquire(blocking=False):  # exactly one line
            if note:
                for key in ("save_async", "raw_GBps", "workdir_broadcast", "sequential"):
                    if out[key] is None:
                        out[key] = {"error": note}
            print(json.dumps(out), flush=True)

    def expire():
        emit("side measurement timed out after %.0f s" % args.side_timeout)
        sys.stdout.flush()
        os._exit(0)

    # N > 1: the side measurements include collectives this repo has only rehearsed (RCCL
    # fan-out over xGMI); a crash in one must not take the headline with it, so rank 0 prints
    # the headline line now and the side results as a "bench-side" JSON line on stderr
    side_to_stderr = world > 1
    if side_to_stderr and out is not None:
        for key in ("save_async", "raw_GBps", "workdir_broadcast", "sequential", "preempt_e2e"):
            out[key] = {"deferred": "stderr: bench-side"}
        emit()
    # armed only now: a timer firing before the N > 1 headline would rewrite its markers
    watchdog = threading.Timer(args.side_timeout, expire)
    watchdog.daemon = True
    watchdog.start()

    async_stall = None
    if not args.no_async:  # untimed side measurement: training-stream stall of save_async
        # every rank reaches every collective below, whatever fails locally (no deadlock)
        err, stall, spill = None, 0.0, 0.0
        try:
            ck.save_async().result()  # allocates the HBM snapshot
        except Exception as error:
            err = repr(error)
        barrier()
        if err is None:
            try:
                a0 = time.perf_counter()
                pending = ck.save_async({"async": True})
                if on_gpu:
                    torch.cuda.current_stream(device).synchronize()
                stall = time.perf_counter() - a0
                pending.result()
                spill = time.perf_counter() - a0
            except Exception as error:
                err = repr(error)
        failed = allmax(1.0 if err else 0.0)
        stall, spill = allmax(stall), allmax(spill)
        async_stall = ({"error": err or "failed on another rank"} if failed else
                       {"stall_ms": round(stall * 1e3, 2), "spill_s": round(spill, 3)})

    raw = None
    if args.codec != "none":  # untimed: the same checkpoint through the codec-free pipeline
        err, rs, rr = None, 0.0, 0.0
        ck.codec = "none"
        try:
            barrier()
            a = time.perf_counter()
            ck.save({"raw": True})
            sync()
            rs = time.perf_counter() - a
            a = time.perf_counter()
            ck.restore()
            sync()
            rr = time.perf_counter() - a
        except Exception as error:
            err = repr(error)
        finally:
            ck.codec = args.codec
        failed = allmax(1.0 if err else 0.0)
        rs, rr = allmax(rs), allmax(rr)
        raw = ({"error": err or "failed on another rank"} if failed else
               {"GBps": round(2 * total / (rs + rr) / 1e9, 3),
                "save_GBps": round(total / rs / 1e9, 3),
                "restore_GBps": round(total / rr / 1e9, 3)})

    sequential = None
    if overlap:  # untimed: the same step with the restore after the save (into the saved tensors)
        err, ss, rr = None, 0.0, 0.0
        try:
            barrier()
            a = time.perf_counter()
            ck.save({"sequential": True})
            sync()
            ss = time.perf_counter() - a
            a = time.perf_counter()
            res = ck.restore()
            sync()
            rr = time.perf_counter() - a
            if res.bad_tiles:
                err = "%d corrupt tiles" % res.bad_tiles
        except Exception as error:
            err = repr(error)
        failed = allmax(1.0 if err else 0.0)
        ss, rr = allmax(ss), allmax(rr)
        sequential = ({"error": err or "failed on another rank"} if failed else
                      {"GBps": round(2 * total / (ss + rr) / 1e9, 3),
                       "save_GBps": round(total / ss / 1e9, 3),
                       "restore_GBps": round(total / rr / 1e9, 3)})

    fanout = None
    # configs 2/3: workdir -> HBM on every rank (untimed; RCCL needs one GPU per rank)
    if args.broadcast_gb > 0 and on_gpu and (world == 1 or backend == "nccl"):
        try:
            import ctypes

            from terraform_provider_iterative_amd.ops import hip
            from terraform_provider_iterative_amd.parallel.fanout import measure_workdir_fanout

            node = ctypes.c_int(-1)
            hip().tpi_device_numa_node(device.index, ctypes.byref(node))
            fanout = measure_workdir_fanout(int(args.broadcast_gb * 1e9), rank, world, device,
                                            barrier, allmax, numa_node=node.value)
        except Exception as error:  # never lose the headline to the side measurement
            fanout = {"error": repr(error)}

    watchdog.cancel()
    e2e = None
    if args.preempt_e2e == "auto" and on_gpu and world == 1:
        # the task's ranks need this process's HBM and host region: give both back first
        ck.close()
        tensors.clear()
        torch.cuda.empty_cache()
        e2e = preempt_e2e(args.total_gb, args.codec, args.e2e_timeout)
    if out is not None and side_to_stderr:
        side = {"save_async": async_stall, "raw_GBps": raw, "workdir_broadcast": fanout,
                "sequential": sequential, "preempt_e2e": e2e,
                "first_log_latency_config2": config2}
        print("bench-side " + json.dumps(side), file=sys.stderr, flush=True)
    elif out is not None:
        out["save_async"] = async_stall
        out["raw_GBps"] = raw
        out["workdir_broadcast"] = fanout
        out["sequential"] = sequential
        out["preempt_e2e"] = e2e
        out["first_log_latency_config2"] = config2
        if isinstance(sequential, dict) and "GBps" in sequential:
            out["value_sequential"] = sequential["GBps"]
    emit()
    ck.close()
    if world > 1:
        dist.destroy_process_group()
    if verified is False:  # a restore that did not rewrite the state is no measurement
        print("bench: restore NOT verified: the restored tensors differ from the saved ones",
              file=sys.stderr, flush=True)
        raise SystemExit(3)


if __name__ == "__main__":
    main()
