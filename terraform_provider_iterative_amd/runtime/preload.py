"""Preloaded successor of a Python rank: an interpreter that has already imported PyTorch and
this package, parked until its rank is preempted, then running the rank's script in-process.

A cold successor spends ~1.8 s of its 1.9 s signal -> restored starting an interpreter and
importing PyTorch (``profiles/round5/r5p/bench.json``, ``preempt_e2e.runs.cold``).  With
``TPI_PRELOAD=1`` the supervisor keeps one of these per rank (``preload_argv`` in its spec,
``csrc/supervisor/supervisor.cpp`` ``keep_preloaded``): spawned with the next incarnation's
environment once the rank has run a while, it imports and then blocks on its activation pipe
(fd ``TPI_STANDBY_FD``, as a warm standby does).  The supervisor activates it at the respawn
("go port=<rendezvous port>"); it then runs the script exactly as ``python script`` would:
``__main__``, ``sys.argv``, ``sys.path[0]`` the script's directory, exit status from
``SystemExit`` or an uncaught exception.  It never touches the GPU before activation (nothing
here initialises HIP unless ``TPI_PRELOAD=gpu``/``gpu-lite``, or -- the default -- until the
supervisor has seen the running incarnation use the GPU from its main process alone: then it
writes "warm" and this process creates its GPU context while parked (``gpu-lite``, ~0.13 s off
the cold recovery); a script whose other processes hold the GPU keeps a plain successor, since
workers it forks before touching the GPU could not use an inherited context).  So the
script's own ``HIP_VISIBLE_DEVICES`` and device choices hold.

The parked process has imported PyTorch before the script runs: environment variables a script
sets before ``import torch`` to configure it (``OMP_NUM_THREADS``, allocator settings) do not
reach a preloaded successor -- set them in the task's ``environment`` block instead, or use
``TPI_PRELOAD=0``.  It waits outside the rank's memory cgroup and joins it when activated.
EOF on the pipe (the rank finished, the task stopped): it exits quietly.

Reference: a spot VM's replacement boots and runs the machine script from the start
(``task/common/machine/machine-script.sh.tpl:89``); here the replacement is a process, and
its start-up is taken off the recovery path.
"""
from __future__ import annotations

import os
import runpy
import sys
import time


def _read_go(fd: int, on_warm=None) -> str:
    """The activation line ("go port=N"; "" at EOF).  A "warm" line before it -- the
    supervisor's evidence that the script uses the GPU from its main process only
    (``supervisor.cpp`` ``check_preload_evidence``) -- calls ``on_warm`` and keeps waiting."""
    data = b""
    while True:
        while b"\n" in data:
            line, data = data.split(b"\n", 1)
            text = line.decode(errors="replace").strip()
            if text == "warm":
                if on_warm is not None:
                    on_warm()
                continue
            return text
        try:
            chunk = os.read(fd, 256)
        except InterruptedError:
            continue
        if not chunk:
            return data.decode(errors="replace").strip()
        data += chunk


def _warm_gpu(engine: bool = True) -> None:
    """``TPI_PRELOAD=gpu``: also initialise the GPU and prewarm a checkpoint engine, as a hot
    standby does (the successor's Checkpointer takes the engine); 2.7 GB of HBM held for the
    life of the rank (``profiles/round5/r5ah/``).  ``gpu-lite`` (``engine=False``, also the
    default's warm-up on evidence): the GPU context, the process's first hardware queue (~137 ms
    of a successor's start, ``profiles/round5/r5z/``) and an engine without its HBM staging
    ring, its hand-off kernels loaded -- all the HBM copy from a live predecessor needs."""
    import torch

    torch.cuda.init()
    torch.empty(1 << 20, dtype=torch.uint8, device="cuda")  # context + caching allocator
    torch.ones(1, device="cuda").add_(1)  # a launch: the first hardware queue and code object
    from terraform_provider_iterative_amd.checkpoint import prewarm_engine

    # gpu-lite: an engine without its staging ring, its hand-off kernels loaded (the HBM copy
    # needs nothing else; a host-path restore allocates the ring at its start)
    prewarm_engine(torch.cuda.current_device(), lite=not engine)
    torch.cuda.synchronize()


def main(argv=None, gpu=False) -> None:
    """``argv``: ``[file.py, args...]`` to run (a shell script's one ``python file.py ...``
    command, :func:`backends.node.shell_python_command`); None: the script path the
    supervisor appends to the command line."""
    argv = list(sys.argv[1:2] if argv is None else argv)
    if not argv:
        raise SystemExit("usage: preload <script> [args...]")
    added = sys.path[0] if sys.path else None  # the package root the launcher put first
    t0 = time.time()
    import torch  # noqa: F401  -- the point: the import a successor would wait for

    import terraform_provider_iterative_amd.checkpoint  # noqa: F401
    from terraform_provider_iterative_amd.checkpoint import preemption
    if gpu:
        try:
            _warm_gpu(engine=gpu != "lite")
        except Exception as error:  # the successor initialises it itself
            print("tpi-preload: GPU warm-up failed: %s" % error, file=sys.stderr, flush=True)
    preloaded_s = time.time() - t0
    fd = int(os.environ.get("TPI_STANDBY_FD", "4"))
    warmed = []

    def warm() -> None:  # the supervisor saw the rank use the GPU from one process only
        if gpu or warmed:
            return
        t1 = time.time()
        try:
            _warm_gpu(engine=False)
            warmed.append(time.time() - t1)
            preemption.journal("preload-gpu-warmed", "GPU context %.3f s" % warmed[0])
        except Exception as error:  # the successor initialises it itself after activation
            print("tpi-preload: GPU warm-up failed: %s" % error, file=sys.stderr, flush=True)
            warmed.append(-1.0)

    line = _read_go(fd, warm)
    try:
        os.close(fd)
    except OSError:
        pass
    if not line.startswith("go"):
        os._exit(0)  # discarded before it was needed
    for token in line.split()[1:]:
        if token.startswith("port="):
            os.environ["MASTER_PORT"] = token[5:]
    for name in ("TPI_STANDBY", "TPI_STANDBY_FD"):
        os.environ.pop(name, None)
    os.environ["TPI_PRELOADED"] = "%.3f" % preloaded_s
    if warmed:
        os.environ["TPI_PRELOAD_GPU_WARMED"] = "%.3f" % warmed[0]
    if os.environ.get("TPI_DEADLINE"):  # set at spawn; the time left is that of now
        try:
            os.environ["TPI_REMAINING_RUN_TIME"] = str(
                max(0, int(float(os.environ["TPI_DEADLINE"]) - time.time())))
        except ValueError:
            pass
    script = os.path.abspath(argv[0])
    # as `python script`: the script's directory first on the path, not the launcher's
    if added is not None and sys.path and sys.path[0] == added:
        sys.path.pop(0)
    if sys.path and sys.path[0] in ("", os.getcwd()):
        sys.path[0] = os.path.dirname(script)
    else:
        sys.path.insert(0, os.path.dirname(script))
    sys.argv = [argv[0]] + argv[1:]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
