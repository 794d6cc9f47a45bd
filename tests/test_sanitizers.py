"""ASan/UBSan builds of the host C++: the native data-plane sources plus a
self-checking harness (tests/native/sanitize_main.cpp), and the rank supervisor driving a
real two-rank task through the node backend."""
import glob
import os
import shutil
import subprocess

import pytest


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
       "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def _compile(out, sources, extra=()):
    cmd = ["g++", "-std=c++17", "-msse4.2", "-pthread", *SAN, *extra, *sources, "-o", out]
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0 and "sanitizer" in res.stdout and "cannot find" in res.stdout:
        pytest.skip("sanitizer runtime not installed")
    assert res.returncode == 0, res.stdout


def test_native_sources_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "sanitize_main")
    srcs = [os.path.join(ROOT, "csrc", "native", f) for f in
            ("filter.cpp", "transfer.cpp", "hostops.cpp", "fileio.cpp", "ctl.cpp")]
    _compile(exe, srcs + [os.path.join(ROOT, "tests", "native", "sanitize_main.cpp")])
    scratch = tmp_path / "scratch"
    scratch.mkdir()
    res = subprocess.run([exe, str(scratch)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         text=True, env=ENV, timeout=300)
    assert res.returncode == 0, res.stdout[-4000:]
    assert "sanitize harness ok" in res.stdout


def test_step_boundary_agreement_under_tsan(tmp_path):
    """The lock-free propose/arrive protocol of csrc/native/ctl.cpp with 8 racing ranks and
    random skew, under ThreadSanitizer: same preemption boundary everywhere, same periodic
    saves, no rank ever past a target, no data race."""
    exe = str(tmp_path / "ctl_stress")
    cmd = ["g++", "-std=c++17", "-pthread", "-fsanitize=thread", "-g", "-O1",
           os.path.join(ROOT, "csrc", "native", "ctl.cpp"),
           os.path.join(ROOT, "tests", "native", "ctl_stress.cpp"), "-o", exe]
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0 and "tsan" in res.stdout.lower() and "cannot find" in res.stdout:
        pytest.skip("ThreadSanitizer runtime not installed")
    assert res.returncode == 0, res.stdout
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    run = [exe, "150", "8"]
    if shutil.which("setarch"):  # TSan's shadow layout wants the classic address space
        run = ["setarch", os.uname().machine, "-R"] + run
    res = subprocess.run(run, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         env=env, timeout=600)
    if "unexpected memory mapping" in res.stdout or "FATAL: ThreadSanitizer" in res.stdout:
        pytest.skip("ThreadSanitizer cannot map its shadow here: " + res.stdout[-300:])
    assert res.returncode == 0, res.stdout[-4000:]
    assert "ctl stress ok" in res.stdout and "WARNING: ThreadSanitizer" not in res.stdout


def test_supervisor_under_asan_ubsan(tmp_path, monkeypatch):
    exe = str(tmp_path / "tpi-supervisor-asan")
    _compile(exe, sorted(glob.glob(os.path.join(ROOT, "csrc", "supervisor", "*.cpp"))))
    monkeypatch.setenv("TPI_SUPERVISOR_BIN", exe)
    monkeypatch.setenv("TPI_MI355X_GPUS", "0,1,2,3")
    monkeypatch.setenv("ASAN_OPTIONS", ENV["ASAN_OPTIONS"])
    from terraform_provider_iterative_amd import backends
    from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
    from terraform_provider_iterative_amd.models.values import Environment, Size, Task
    from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

    state = tmp_path / "state"
    cloud = Cloud(provider="mi355x",
                  credentials=Credentials(node=NodeCredentials(state_root=str(state))))
    spec = Task(size=Size(machine="m+mi355x"), parallelism=2,
                environment=Environment(script="#!/bin/sh\necho rank $RANK of $WORLD_SIZE\n"
                                               "seq 1 2000\n", timeout=60))
    task = backends.new(cloud, new_deterministic_identifier("asan-sup"), spec)
    task.create()
    try:
        status = task.wait(60)
        assert status["succeeded"] == 2, status
        logs = task.logs()
        assert len(logs) == 2 and all("rank" in log and "2000" in log for log in logs)
        reports = []
        for dirpath, _, files in os.walk(str(state)):
            reports += [os.path.join(dirpath, f) for f in files if f == "supervisor.log"]
        assert reports
        for path in reports:
            text = open(path, errors="replace").read()
            for marker in ("AddressSanitizer", "LeakSanitizer", "runtime error"):
                assert marker not in text, text[-2000:]
    finally:
        task.delete()


def test_supervisor_preemption_paths_under_asan_ubsan(tmp_path, monkeypatch):
    # gang of 2 ranks: leo preempt -> spill -> "released" hand-off -> warm standbys activated
    import sys
    import time

    from test_preemption import ROOT as _root, STANDBY

    exe = str(tmp_path / "tpi-supervisor-asan")
    _compile(exe, sorted(glob.glob(os.path.join(ROOT, "csrc", "supervisor", "*.cpp"))))
    monkeypatch.setenv("TPI_SUPERVISOR_BIN", exe)
    monkeypatch.setenv("TPI_WARM_STANDBY", "1")
    monkeypatch.setenv("ASAN_OPTIONS", ENV["ASAN_OPTIONS"])
    from terraform_provider_iterative_amd import backends
    from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
    from terraform_provider_iterative_amd.models.values import Environment, Task, Variables
    from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier

    script = STANDBY.replace('".spill")', '".spill" + os.environ["RANK"])') % {
        "python": sys.executable, "root": _root, "steps": 30}
    state = tmp_path / "state"
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(state))))
    spec = Task(parallelism=2, environment=Environment(
        script=script, timeout=120, variables=Variables({"TPI_TASK": "true"})))
    task = backends.new(cloud, new_deterministic_identifier("asan-preempt"), spec)
    task.create()
    try:
        deadline = time.time() + 60
        while time.time() < deadline and sum("step 3" in l for l in task.logs()) < 2:
            time.sleep(0.05)
        task.preempt()
        status = task.wait(90)
        logs = task.logs()
        assert status["succeeded"] == 2 and status["failed"] == 0, (status, logs)
        assert sum("activated" in l and "final 30 30" in l for l in logs) == 2, logs
        codes = [e.code for e in task.events()]
        assert codes.count("rank-released") == 2 and codes.count("standby-activated") == 2
        for dirpath, _, files in os.walk(str(state)):
            for f in files:
                if f == "supervisor.log":
                    text = open(os.path.join(dirpath, f), errors="replace").read()
                    for marker in ("AddressSanitizer", "LeakSanitizer", "runtime error"):
                        assert marker not in text, text[-2000:]
    finally:
        task.delete()


def test_stager_under_asan_ubsan(tmp_path, monkeypatch):
    """csrc/stager/stager.cpp (host code) built with ASan/UBSan by ROCm's clang and linked to
    the production libtpi_hip.so; then the host-mode staging flow of tests/test_stage.py
    (3 ranks, sharded fan-out, attach, dirty-shard write-back) runs on it."""
    import sys

    from terraform_provider_iterative_amd import _build

    clang = "/opt/rocm/llvm/bin/clang++"
    if not os.path.exists(clang):
        pytest.skip("ROCm clang not installed")
    _build.build_stager()  # builds libtpi_hip.so too
    exe = str(tmp_path / "tpi-stager-asan")
    tl = _build.torch_lib_dir()
    cmd = [clang, "-std=c++17", "-pthread", *SAN, "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", os.path.join(ROOT, "csrc", "stager", "stager.cpp"),
           "-L" + _build.LIB, "-ltpi_hip", "-Wl,-rpath," + _build.LIB, "-L" + tl,
           "-Wl,-rpath," + tl, "-lamdhip64", "-o", exe]
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0 and "cannot find" in res.stdout and "rt" in res.stdout:
        pytest.skip("sanitizer runtime not installed")
    assert res.returncode == 0, res.stdout[-3000:]
    # the HIP runtime's own allocations are not ours to audit: leaks off, errors fatal
    monkeypatch.setenv("ASAN_OPTIONS", "detect_leaks=0:halt_on_error=1:abort_on_error=0")
    monkeypatch.setenv("UBSAN_OPTIONS", ENV["UBSAN_OPTIONS"])
    monkeypatch.setenv("TPI_STAGER_BIN", exe)
    monkeypatch.setenv("TPI_MI355X_GPUS", "0,1,2,3,4,5,6,7")
    monkeypatch.setenv("PYTHONPATH", ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_stage import ATTACH, _task, _workdir

    from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials

    cloud = Cloud(provider="mi355x", credentials=Credentials(
        node=NodeCredentials(state_root=str(tmp_path / "st"))))
    work, sizes = _workdir(tmp_path)
    task = _task(cloud, "asan-stage", ATTACH, work, parallelism=3,
                 env={"TPI_STAGE": "host", "TPI_STAGE_METHOD": "sharded",
                      "TPI_SYNC_INTERVAL": "0.2"})
    task.create()
    try:
        status = task.wait(120)
        log = open(os.path.join(task.sup_dir, "stager.log"), errors="replace").read()
        for marker in ("AddressSanitizer", "runtime error", "UndefinedBehaviorSanitizer"):
            assert marker not in log, log[-3000:]
        assert status["succeeded"] == 3, (task.logs(), log[-2000:])
        data = open(os.path.join(task.data_dir, "a.bin"), "rb").read()
        assert data[:3] == b"XYZ" and len(data) == sizes["a.bin"]
    finally:
        task.delete()


def test_supervisor_hand_off_protocol_under_asan_ubsan(tmp_path, monkeypatch):
    """The round-4 supervisor paths under ASan/UBSan: the notify line protocol (`released`,
    `restored hbm`, `closed`), SIGUSR2 on close, exit tracing from /proc, resources released
    before a slow released process is reaped, and the memory cgroup set-up."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_handoff_protocol import test_predecessor_released_only_after_closed

    exe = str(tmp_path / "tpi-supervisor-asan")
    _compile(exe, sorted(glob.glob(os.path.join(ROOT, "csrc", "supervisor", "*.cpp"))))
    monkeypatch.setenv("ASAN_OPTIONS", ENV["ASAN_OPTIONS"])
    monkeypatch.setenv("UBSAN_OPTIONS", ENV["UBSAN_OPTIONS"])
    for die in (False, True):
        run = tmp_path / ("die" if die else "closed")
        run.mkdir()
        test_predecessor_released_only_after_closed(exe, run, die)
