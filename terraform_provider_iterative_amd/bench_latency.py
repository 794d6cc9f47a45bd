"""apply -> first-log latency of an ``iterative_task`` on the node runtime (BASELINE metric).

Two measurements, both from a fresh state root and a hello-world ``main.tf``:

* ``cli``: wall time from launching ``tpi apply -auto-approve`` (a new Python process, as a
  user would) until the first line of the task's log is on disk;
* ``api``: the same from calling the resource's Create in-process.

The reference's floor for the same metric is VM provisioning + tool downloads + the 5 s log
tick (machine-script.sh.tpl:108-116) + the 3 s ``leo read`` poll (read.go:124).
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from typing import Dict, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MAIN_TF = '''
resource "iterative_task" "latency" {
  name    = "latency-%(tag)s"
  cloud   = "%(cloud)s"
  machine = "%(machine)s"
  parallelism = %(parallelism)d
  storage {
    workdir = "."
  }
  script = <<-END
    #!/bin/sh
    echo "first log line"
  END
}
'''


def _first_log(state_root: str, timeout: float, t0: float, poll: float = 0.0005,
               count: int = 1, proc: Optional[subprocess.Popen] = None) -> Optional[float]:
    """Seconds from ``t0`` until ``count`` ranks' logs (``reports/task-*``) hold a line;
    None at the timeout, or at once when ``proc`` (the apply) has failed."""
    pattern = os.path.join(state_root, "*", "*", "reports", "task-*")
    deadline = t0 + timeout
    while time.perf_counter() < deadline:
        if proc is not None and proc.poll() not in (None, 0):
            return None
        seen = 0
        for path in glob.glob(pattern):
            try:
                seen += os.path.getsize(path) > 0
            except OSError:
                pass
        if seen >= count:
            return time.perf_counter() - t0
        time.sleep(poll)
    return None


def _gate_wait(state_root: str) -> float:
    """Seconds the task's start waited for its GPUs' memory (``gpu-drain`` events: the driver
    still wiping memory an earlier process freed), summed over the task's journals -- part of
    the measured latency, reported beside it."""
    waited = 0.0
    for path in glob.glob(os.path.join(state_root, "*", "*", "supervisor", "events.jsonl")):
        try:
            with open(path) as handle:
                for line in handle:
                    if '"gpu-drain"' not in line:
                        continue
                    for item in json.loads(line).get("description", []):
                        if isinstance(item, str) and item.startswith("waited "):
                            waited += float(item.split()[1])
        except (OSError, ValueError):
            continue
    return waited


def _cleanup(workdir: str, env: Dict[str, str]) -> None:
    subprocess.run([sys.executable, os.path.join(ROOT, "bin", "tpi"), "destroy", "-auto-approve"],
                   cwd=workdir, env=env, capture_output=True, timeout=120)


def measure_first_log_latency(timeout: float = 60.0, cloud: Optional[str] = None,
                              repeats: int = 3, parallelism: int = 1) -> Dict[str, float]:
    """Returns ``{"cli_s": .., "api_s": .., "cloud": .., "gpu_drain_max_s": ..}`` (medians over
    ``repeats``; the last: the longest wait of any sample's start for its GPUs' memory, included
    in its latency): the first log line of any rank; with ``parallelism`` N > 1 also ``cli_all_s`` / ``api_all_s``,
    until every one of the N ranks (one GPU each on ``mi355x``) has logged."""
    gpu = False
    try:
        import torch

        gpu = torch.cuda.is_available()
    except ImportError:  # pragma: no cover
        pass
    cloud = cloud or ("mi355x" if gpu else "local")
    machine = "m+mi355x" if cloud == "mi355x" else "s"
    cli, api, cli_all, api_all, gate = [], [], [], [], []
    for i in range(repeats):
        base = tempfile.mkdtemp(prefix="tpi-latency-")
        try:
            work = os.path.join(base, "work")
            os.makedirs(work)
            with open(os.path.join(work, "main.tf"), "w") as handle:
                handle.write(MAIN_TF % {"tag": "%d%d" % (os.getpid(), i), "cloud": cloud,
                                        "machine": machine, "parallelism": parallelism})
            env = dict(os.environ)
            env["TPI_STATE_ROOT"] = os.path.join(base, "state")
            env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
            t0 = time.perf_counter()
            proc = subprocess.Popen([sys.executable, os.path.join(ROOT, "bin", "tpi"), "apply",
                                     "-auto-approve"], cwd=work, env=env,
                                    stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            latency = _first_log(env["TPI_STATE_ROOT"], timeout, t0, proc=proc)
            every = _first_log(env["TPI_STATE_ROOT"], timeout, t0, count=parallelism, proc=proc)
            proc.wait(timeout=timeout)
            gate.append(_gate_wait(env["TPI_STATE_ROOT"]))
            if latency is not None:
                cli.append(latency)
            if every is not None:
                cli_all.append(every)
            _cleanup(work, env)
            # in-process API path
            from .provider import resources
            from .models.schema import normalize

            old = os.environ.get("TPI_STATE_ROOT")
            os.environ["TPI_STATE_ROOT"] = os.path.join(base, "state-api")
            cwd = os.getcwd()
            os.chdir(work)
            try:
                data = normalize("iterative_task", {
                    "name": "latency-api-%d%d" % (os.getpid(), i), "cloud": cloud,
                    "machine": machine, "storage": [{"workdir": "."}],
                    "parallelism": parallelism,
                    "script": "#!/bin/sh\necho first log line\n"})
                t1 = time.perf_counter()
                result = resources.task_create(data)
                created = bool(result.id) and not any(
                    d.severity == "error" for d in result.diagnostics)
                wait = timeout if created else 0.0  # a refused create logs nothing
                lat = _first_log(os.environ["TPI_STATE_ROOT"], wait, t1)
                every = _first_log(os.environ["TPI_STATE_ROOT"], wait, t1, count=parallelism)
                gate.append(_gate_wait(os.environ["TPI_STATE_ROOT"]))
                if lat is not None:
                    api.append(lat)
                if every is not None:
                    api_all.append(every)
                if result.id:
                    data["id"] = result.id
                    resources.task_delete(data)
            finally:
                os.chdir(cwd)
                if old is None:
                    os.environ.pop("TPI_STATE_ROOT", None)
                else:
                    os.environ["TPI_STATE_ROOT"] = old
        finally:
            shutil.rmtree(base, ignore_errors=True)

    def median(xs):
        xs = sorted(xs)
        return round(xs[len(xs) // 2], 4) if xs else None

    out = {"cli_s": median(cli), "api_s": median(api), "cloud": cloud, "samples": len(cli),
           "parallelism": parallelism,
           # the most any sample's start waited for the driver to give its GPUs' memory back
           # (0 on an idle node; after a job that freed 100+ GB, seconds: gpu-drain)
           "gpu_drain_max_s": round(max(gate), 4) if gate else None}
    if parallelism > 1:
        out.update(cli_all_s=median(cli_all), api_all_s=median(api_all))
    return out


if __name__ == "__main__":
    print(json.dumps(measure_first_log_latency()))
