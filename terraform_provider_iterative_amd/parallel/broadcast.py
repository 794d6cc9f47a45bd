"""Fan-out of one rank's buffer to every rank of a task.

The reference lets each of ``parallelism`` machines download the workdir from the bucket on
its own (``machine-script.sh.tpl:89``).  On one MI355X node the ranks sit on GPUs joined by
point-to-point xGMI links (7 x ~153 GB/s per GPU on the 8-GPU platform), so the workdir is
read from host memory once and fanned out GPU-to-GPU with RCCL (``torch.distributed``,
backend ``nccl`` = RCCL):

* ``broadcast``           one ``ncclBroadcast`` (pipelined over RCCL's channels);
* ``scatter_allgather``   the root sends rank i its 1/N slice over the i-th link in parallel
                          (grouped P2P), then an in-place all-gather rebuilds the buffer
                          everywhere -- every rank's links carry traffic instead of the
                          root's outgoing ring edge bounding the whole transfer;
* ``auto``                ``broadcast`` for 2 ranks, ``scatter_allgather`` above.

Works with ``gloo`` too (CPU tensors), which is how the tests exercise it.
"""
from __future__ import annotations

import time
from typing import Optional

METHODS = ("broadcast", "scatter_allgather", "auto")


def _dist():
    import torch.distributed as dist

    return dist


def choose_method(world: int, method: str = "auto") -> str:
    if method not in METHODS:
        raise ValueError("unknown broadcast method %r" % method)
    if method != "auto":
        return method
    return "broadcast" if world <= 2 else "scatter_allgather"


def broadcast_buffer(buf, src: int = 0, group=None, method: str = "auto") -> float:
    """Make ``buf`` (1-D uint8 tensor, same length on every rank) equal to ``src``'s copy.

    Returns the wall time in seconds (synchronised on device buffers).
    """
    dist = _dist()
    import torch

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1 or buf.numel() == 0:
        return 0.0
    on_device = buf.device.type == "cuda"
    t0 = time.perf_counter()
    method = choose_method(world, method)
    if method == "broadcast":
        dist.broadcast(buf, src=_global(src, group), group=group)
    else:
        n = buf.numel()
        shard = (n + world - 1) // world
        # Work on a padded view only when needed (the padding never leaves the device).
        padded = buf if shard * world == n else torch.zeros(shard * world, dtype=buf.dtype,
                                                             device=buf.device)
        if padded is not buf and rank == src:
            padded[:n].copy_(buf)
        shards = padded.view(world, shard)
        ops = []
        if rank == src:
            for r in range(world):
                if r != src:
                    ops.append(dist.P2POp(dist.isend, shards[r], _global(r, group), group))
        else:
            ops.append(dist.P2POp(dist.irecv, shards[rank], _global(src, group), group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        allgather_inplace(padded, group)
        if padded is not buf:
            buf.copy_(padded[:n])
    if on_device:
        torch.cuda.synchronize(buf.device)
    return time.perf_counter() - t0


def allgather_inplace(padded, group=None) -> None:
    """In-place all-gather of ``padded`` viewed as ``world`` equal shards: rank r's shard r
    is kept, every other shard is filled from its owner.  RCCL takes the single-buffer
    ``all_gather_into_tensor`` (one ring pass, no staging copy); gloo lacks it, so there
    the list form gathers into scratch tensors that are copied back into the views."""
    import torch

    dist = _dist()
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    shards = padded.view(world, -1)
    if padded.device.type == "cuda":
        dist.all_gather_into_tensor(padded, shards[rank], group=group)
        return
    tmp = [torch.empty_like(shards[r]) for r in range(world)]
    dist.all_gather(tmp, shards[rank].clone(), group=group)
    for r in range(world):
        if r != rank:
            shards[r].copy_(tmp[r])


def _global(rank: int, group) -> int:
    if group is None:
        return rank
    dist = _dist()
    return dist.get_global_rank(group, rank)


def measure(nbytes: int, method: str = "auto", iters: int = 3, warmup: int = 1,
            device=None, group=None) -> Optional[dict]:
    """Broadcast bandwidth benchmark (config 3); returns GB/s as seen by the receivers."""
    import torch

    dist = _dist()
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return None
    buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
    if dist.get_rank(group) == 0:
        buf.fill_(7)
    times = []
    for i in range(warmup + iters):
        dist.barrier(group=group)
        t = broadcast_buffer(buf, 0, group, method)
        if i >= warmup:
            times.append(t)
    ok = bool((buf[:: max(1, nbytes // 4096)] == 7).all().item())
    t = max(times)
    worst = torch.tensor([t], dtype=torch.float64, device=device)
    dist.all_reduce(worst, op=dist.ReduceOp.MAX, group=group)
    t = float(worst.item())
    return {"method": choose_method(dist.get_world_size(group), method), "bytes": nbytes,
            "seconds": t, "GBps": nbytes / t / 1e9 if t > 0 else None, "verified": ok}


def measure_independent_h2d(nbytes: int, iters: int = 3, warmup: int = 1, device=None,
                            group=None, chunk: int = 2 << 30) -> Optional[dict]:
    """The reference's fan-out analogue: every rank pulls its own copy of the ``nbytes``
    workdir from host memory (each VM's ``rclone copy``, ``machine-script.sh.tpl:89``) --
    concurrent H2D over every GPU's PCIe link from pinned host DRAM, ``chunk`` bytes at a
    time.  Same return shape as :func:`measure`, for comparison with the xGMI fan-out."""
    import torch

    dist = _dist()
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return None
    chunk = min(chunk, nbytes)
    host = torch.full((chunk,), 7, dtype=torch.uint8).pin_memory()
    buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
    times = []
    for i in range(warmup + iters):
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for lo in range(0, nbytes, chunk):
            n = min(chunk, nbytes - lo)
            buf[lo:lo + n].copy_(host[:n], non_blocking=True)
        torch.cuda.synchronize(buf.device)
        if i >= warmup:
            times.append(time.perf_counter() - t0)
    ok = bool((buf[:: max(1, nbytes // 4096)] == 7).all().item())
    worst = torch.tensor([max(times)], dtype=torch.float64, device=device)
    dist.all_reduce(worst, op=dist.ReduceOp.MAX, group=group)
    t = float(worst.item())
    return {"method": "independent_h2d", "bytes": nbytes, "seconds": t,
            "GBps": nbytes / t / 1e9 if t > 0 else None, "verified": ok}
