"""Config 3 measurement: a task's workdir from the page cache into HBM on every rank.

The same native pieces the runtime's stager uses (``runtime.stage.Loader`` +
``parallel.comm.TaskComm``), driven from one process per GPU (bench.py's ranks), for the
three schedules:

* ``sharded``      rank i loads the i-th 1/N of the image over its own PCIe link, then one
                   in-place all-gather over xGMI (the runtime default);
* ``broadcast``    rank 0 loads the whole image, then an RCCL broadcast;
* ``independent``  every rank loads the whole image itself -- the reference's pattern, where
                   each machine runs its own ``rclone copy`` (machine-script.sh.tpl:89).

Every method is timed from a barrier to the last rank's completion, and every rank's copy is
checked against rank 0's with the shard-hash kernel.
"""
from __future__ import annotations

import os
import shutil
import time
from typing import Callable, Dict, Optional

METHODS = ("sharded", "broadcast", "independent")


def write_workdir(path: str, nbytes: int, nfiles: int = 10, block: int = 256 << 20) -> None:
    """``nfiles`` files totalling ``nbytes`` of random-looking data (a random block reused
    with a per-file prefix; content does not matter to a DMA)."""
    import numpy as np

    os.makedirs(path, exist_ok=True)
    rng = np.random.default_rng(3)
    blob = rng.integers(0, 256, min(block, max(nbytes, 1)), dtype=np.uint8).tobytes()
    per = nbytes // nfiles
    for i in range(nfiles):
        size = per if i < nfiles - 1 else nbytes - per * (nfiles - 1)
        with open(os.path.join(path, "shard-%03d.bin" % i), "wb") as handle:
            handle.write(("file %d\n" % i).encode())
            left = size - handle.tell()
            while left > 0:
                n = min(left, len(blob))
                handle.write(blob[:n])
                left -= n


XGMI_LINK_GBPS = 153.0  # one MI355X xGMI link, per direction (7 per GPU on an 8-GPU node)


def measure_workdir_fanout(nbytes: int, rank: int, world: int, device, barrier: Callable,
                           allmax: Callable[[float], float], workdir: Optional[str] = None,
                           methods=METHODS, numa_node: int = -1) -> Dict[str, dict]:
    import torch
    import torch.distributed as dist

    from ..ops import shard_hash
    from ..runtime.stage import ALIGN, Loader, layout
    from .comm import TaskComm

    workdir = workdir or os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                      "tpi-fanout-%s" % os.environ.get("MASTER_PORT", "0"))
    requested = nbytes
    if rank == 0:  # a small TMPDIR shrinks the workdir instead of failing the measurement
        parent = os.path.dirname(os.path.abspath(workdir))
        try:
            free = shutil.disk_usage(parent).free
        except OSError:
            free = 0
        nbytes = int(min(nbytes, max(0, 0.4 * free)))
    nbytes = int(allmax(float(nbytes) if rank == 0 else 0.0))
    if nbytes < (64 << 20):
        raise RuntimeError("no room for a synthetic workdir under %s" % workdir)
    err = None
    if rank == 0:
        try:
            write_workdir(workdir, nbytes)
        except OSError as error:  # every rank must learn it, no deadlock
            err = error
            shutil.rmtree(workdir, ignore_errors=True)
    barrier()
    if allmax(1.0 if err else 0.0):
        raise RuntimeError("cannot write the synthetic workdir: %s" % (err or "on rank 0"))
    files, size = layout(workdir)
    quantum = ALIGN * world
    total = (size + quantum - 1) // quantum * quantum
    image = torch.empty(total, dtype=torch.uint8, device=device)
    comm = TaskComm.from_group(device=device.index) if world > 1 else None
    out: Dict[str, dict] = {"bytes": total, "files": len(files),
                            "requested_bytes": requested,
                            # the RCCL communicator the runtime built over the task's ranks
                            "task_comm_world": comm.world if comm is not None else 1}
    try:
        with Loader(device.index, chunk_bytes=64 << 20, nbuf=4, threads=16,
                    numa_node=numa_node) as loader:
            loader.load(workdir, files, 0, min(total, 256 << 20), image.data_ptr())  # warm
            for method in methods:
                if world == 1 and method != "sharded":
                    continue
                image.zero_()
                barrier()
                t0 = time.perf_counter()
                if method == "sharded":
                    shard = total // world
                    loader.load(workdir, files, rank * shard, (rank + 1) * shard,
                                image.data_ptr())
                    torch.cuda.synchronize(device)
                    t1 = time.perf_counter()
                    if comm is not None:
                        barrier()  # time the all-gather alone, all ranks' shards loaded
                        ta = time.perf_counter()
                        comm.allgather_inplace(image, shard)
                        gather_s = allmax(time.perf_counter() - ta)
                elif method == "broadcast":
                    if rank == 0:
                        loader.load(workdir, files, 0, total, image.data_ptr())
                    t1 = time.perf_counter()
                    comm.broadcast(image, total, root=0)
                else:
                    loader.load(workdir, files, 0, total, image.data_ptr())
                    t1 = time.perf_counter()
                torch.cuda.synchronize(device)
                t2 = time.perf_counter()
                load_s, elapsed = allmax(t1 - t0), allmax(t2 - t0)
                mine = shard_hash(image)
                verified = True
                if world > 1:
                    ref = mine.clone()
                    dist.broadcast(ref, src=0)
                    ok = torch.tensor([float(torch.equal(mine, ref))], device=device)
                    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                    verified = bool(ok.item() == 1.0)
                out[method] = {"s": round(elapsed, 4), "load_s": round(load_s, 4),
                               "GBps_per_rank": round(total / elapsed / 1e9, 2),
                               "GBps_aggregate": round(world * total / elapsed / 1e9, 2),
                               "verified": verified}
                if method == "sharded" and comm is not None:
                    # all-gather bus bandwidth (each rank receives (N-1)/N of the image), next
                    # to what one xGMI link carries: a single ring is bound by it, so a bus
                    # rate above it means RCCL spread the rings over several links
                    busbw = total * (world - 1) / world / gather_s / 1e9
                    out[method].update({"allgather_s": round(gather_s, 4),
                                        "allgather_busbw_GBps": round(busbw, 2),
                                        "xgmi_link_GBps": XGMI_LINK_GBPS,
                                        "busbw_over_one_link": round(busbw / XGMI_LINK_GBPS, 2)})
    finally:
        if comm is not None:
            comm.close()
        del image
        barrier()
        if rank == 0:
            shutil.rmtree(workdir, ignore_errors=True)
    return out
