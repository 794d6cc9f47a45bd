"""The rank supervisor (csrc/supervisor/supervisor.cpp) driven directly through spec.json.

Covers the scaling-group / machine-script semantics it replaces: fail-fast of a coupled
group (k8s Job with parallelism), restart limits (BackoffLimit), gang vs independent respawn
after preemption (ASG/MIG respawn), deadline before start (``sleep infinity`` past the
deadline, machine-script.sh.tpl:36-41), stop = scale to zero without status
(machine-script.sh.tpl:10-15,51), and faithful log capture.
"""
import json
import os
import signal
import subprocess
import time

import pytest

from terraform_provider_iterative_amd import _build


@pytest.fixture(scope="module")
def binary():
    return _build.build_supervisor()


def _spec(tmp_path, script, parallelism=1, **extra):
    task = tmp_path / "task"
    for d in ("data", "reports", "supervisor"):
        (task / d).mkdir(parents=True, exist_ok=True)
    path = task / "supervisor" / "script"
    path.write_text(script)
    path.chmod(0o755)
    spec = {"task_id": "tpi-sup-test", "task_dir": str(task), "workdir": str(task / "data"),
            "script": str(path), "env": {"PATH": os.environ["PATH"]},
            "parallelism": parallelism, "ranks": [{"gpus": "", "rank_gpus": ""}] * parallelism,
            "grace_seconds": 5, "master_port": 29999}
    spec.update(extra)
    spec_path = task / "supervisor" / "spec.json"
    spec_path.write_text(json.dumps(spec))
    return task, str(spec_path)


def _run(binary, spec_path, timeout=60):
    return subprocess.run([binary, spec_path], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                          timeout=timeout)


def _statuses(task):
    out = {}
    for name in sorted(os.listdir(task / "reports")):
        if name.startswith("status-"):
            out[name] = json.loads((task / "reports" / name).read_text())
    return out


def _events(task):
    with open(task / "supervisor" / "events.jsonl") as handle:
        return [json.loads(line) for line in handle if line.strip()]


def _logs(task):
    return [(task / "reports" / n).read_text() for n in sorted(os.listdir(task / "reports"))
            if n.startswith("task-")]


def test_fail_fast_stops_the_group(binary, tmp_path):
    script = '#!/bin/sh\nif [ "$RANK" = 1 ]; then echo bad; exit 3; fi\nsleep 30\n'
    task, spec = _spec(tmp_path, script, parallelism=3, fail_fast=True)
    t0 = time.time()
    _run(binary, spec)
    assert time.time() - t0 < 15
    results = sorted((s["result"], s["code"]) for s in _statuses(task).values())
    assert ("exit-code", "3") in results
    assert sum(1 for r, _ in results if r == "signal") == 2


def test_restart_limit(binary, tmp_path):
    # every incarnation "gets preempted" (exit 143): respawned until max_restarts
    task, spec = _spec(tmp_path, "#!/bin/sh\necho run $TPI_RESTART_COUNT\nexit 143\n",
                       max_restarts=2)
    _run(binary, spec)
    codes = [e["code"] for e in _events(task)]
    assert codes.count("respawn") == 2 and "rank-restart-limit" in codes
    statuses = list(_statuses(task).values())
    assert [s["result"] for s in statuses] == ["start-limit-hit"]
    logs = "".join(_logs(task))
    assert "run 0" in logs and "run 1" in logs and "run 2" in logs


@pytest.mark.parametrize("gang", [True, False])
def test_gang_and_independent_respawn(binary, tmp_path, gang):
    script = ('#!/bin/sh\n'
              'if [ "$RANK" = 0 ] && [ "$TPI_RESTART_COUNT" = 0 ]; then exit 143; fi\n'
              'if [ "$RANK" = 1 ] && [ "$TPI_RESTART_COUNT" = 0 ]; then sleep 2; fi\n'
              'echo "rank $RANK restart $TPI_RESTART_COUNT"\n')
    task, spec = _spec(tmp_path, script, parallelism=2, gang=gang, fail_fast=False)
    _run(binary, spec)
    respawned = sorted(int(e["description"][0].split()[1]) for e in _events(task)
                       if e["code"] == "respawn")
    assert respawned == ([0, 1] if gang else [0])
    statuses = _statuses(task)
    assert sum(1 for s in statuses.values() if s["result"] == "success") == 2
    # a rank killed for the gang restart writes no status, like a preempted machine
    assert len(statuses) == 2


def test_deadline_in_the_past(binary, tmp_path):
    task, spec = _spec(tmp_path, "#!/bin/sh\necho never\n", parallelism=2,
                       deadline=time.time() - 10)
    _run(binary, spec)
    statuses = list(_statuses(task).values())
    assert len(statuses) == 2 and all(s["result"] == "timeout" for s in statuses)
    assert "never" not in "".join(_logs(task))


def test_deadline_kills_running_rank(binary, tmp_path):
    task, spec = _spec(tmp_path, "#!/bin/sh\necho start\nsleep 60\n", deadline=time.time() + 1.5)
    t0 = time.time()
    _run(binary, spec)
    assert time.time() - t0 < 15
    (status,) = _statuses(task).values()
    assert status["result"] == "timeout"


def test_stop_scales_to_zero_without_status(binary, tmp_path):
    task, spec = _spec(tmp_path, "#!/bin/sh\necho up\nsleep 60\n", parallelism=2)
    proc = subprocess.Popen([binary, spec], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        deadline = time.time() + 20
        while time.time() < deadline and "up" not in "".join(_logs(task)).split():
            time.sleep(0.05)
        proc.send_signal(signal.SIGTERM)
        proc.wait(timeout=20)
    finally:
        if proc.poll() is None:
            proc.kill()
    assert _statuses(task) == {}
    codes = [e["code"] for e in _events(task)]
    assert "stop-requested" in codes and codes.count("rank-stopped") == 2


def test_log_capture_is_faithful(binary, tmp_path):
    script = ('#!/bin/sh\n'
              'printf "first\\n"\n'
              'echo "to stderr" 1>&2\n'
              'head -c 200000 /dev/zero | tr "\\0" x\n'   # one 200 KB line
              'printf "\\n"\n'
              'printf "tab\\there\\n"\n'
              'printf "no newline at end"\n')
    task, spec = _spec(tmp_path, script)
    _run(binary, spec)
    (log,) = _logs(task)
    lines = log.splitlines()
    messages = [line.split(" ", 1)[1] if " " in line else "" for line in lines]
    assert messages[0] == "first"
    assert "to stderr" in messages
    assert "x" * 200000 in messages
    assert "tab\there" in messages
    assert messages[-1] == "no newline at end"
    stamp = lines[0].split(" ", 1)[0]
    assert len(stamp) == 20 and stamp.endswith("Z") and stamp[10] == "T"
    (status,) = _statuses(task).values()
    assert status == {"result": "success", "code": "0", "status": "exited"}


def test_rank_cpu_affinity_from_spec(binary, tmp_path):
    # the NUMA-local cores placed for a rank become its affinity mask (children inherit it)
    allowed = sorted(os.sched_getaffinity(0))
    want = allowed[:1]
    task, spec = _spec(tmp_path, "#!/bin/sh\ngrep Cpus_allowed_list /proc/self/status\n",
                       parallelism=2,
                       ranks=[{"gpus": "", "rank_gpus": "", "cpus": want},
                              {"gpus": "", "rank_gpus": ""}])
    assert _run(binary, spec).returncode == 0
    logs = _logs(task)
    lines = sorted(l.split("\t")[-1].strip() for log in logs for l in log.splitlines() if l)
    full = ",".join(map(str, allowed))
    assert str(want[0]) in lines
    assert len(lines) == 2 and any(l != str(want[0]) or full == str(want[0]) for l in lines)


def test_supervisor_takes_the_first_free_rendezvous_port(binary, tmp_path):
    """``master_port_probe``: the spec's port is a base, and the supervisor (not ``tpi
    apply``) takes the first port from it that binds -- journalled when it is not the base."""
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as busy:
        busy.bind(("127.0.0.1", 0))
        base = busy.getsockname()[1]
        busy.listen(1)
        task, spec = _spec(tmp_path, "#!/bin/sh\necho port=$MASTER_PORT\n", master_port=base,
                           master_port_probe=True)
        _run(binary, spec)
    port = int(_logs(task)[0].split("port=")[1].split()[0])
    assert base < port <= base + 255
    assert any(e["code"] == "rendezvous" and "master port %d" % port in e["description"]
               for e in _events(task))
    # a free base is used as it is, without a journal line
    task2, spec2 = _spec(tmp_path / "again", "#!/bin/sh\necho port=$MASTER_PORT\n",
                         master_port=port, master_port_probe=True)
    _run(binary, spec2)
    assert "port=%d" % port in _logs(task2)[0]
    assert not any(e["code"] == "rendezvous" for e in _events(task2))
