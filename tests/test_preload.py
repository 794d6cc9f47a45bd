"""Preloaded successors (``TPI_PRELOAD=1``, ``runtime/preload.py`` + the supervisor's
``keep_preloaded``): a Python rank's successor has imported PyTorch before the preemption and
then runs the script exactly as ``python script`` would.

Reference: the replacement of a preempted spot VM runs the machine script from the start
(``task/common/machine/machine-script.sh.tpl:89``).
"""
import os
import sys
import time

from terraform_provider_iterative_amd import backends
from terraform_provider_iterative_amd.backends.node import shebang_python
from terraform_provider_iterative_amd.models.cloud import Cloud, Credentials, NodeCredentials
from terraform_provider_iterative_amd.models.values import Environment, Task, Variables
from terraform_provider_iterative_amd.utils.identifier import new_deterministic_identifier


def test_only_scripts_of_this_interpreter_are_preloaded():
    exe = sys.executable
    assert shebang_python("#!%s\nprint(1)\n" % exe) == (exe, [])
    assert shebang_python("#!%s -u\n" % exe) == (exe, ["-u"])
    assert shebang_python("#!/bin/bash\necho hi\n") is None
    assert shebang_python("print(1)\n") is None
    assert shebang_python("#!%s -m mod\n" % exe) is None  # not a plain script run
    assert shebang_python("#!/nonexistent/python3\n") is None
    env_form = shebang_python("#!/usr/bin/env %s\n" % os.path.basename(exe))
    import shutil

    found = shutil.which(os.path.basename(exe))
    if found and os.path.realpath(found) == os.path.realpath(exe):
        assert env_form == (found, [])
    else:
        assert env_form is None


def test_a_virtualenv_interpreter_is_launched_as_named(tmp_path):
    """A venv's python is a link to the same binary; the preloaded successor must start it by
    that path, or the venv's site-packages would be missing."""
    venv = tmp_path / "venv" / "bin"
    venv.mkdir(parents=True)
    link = venv / "python3"
    link.symlink_to(os.path.realpath(sys.executable))
    assert shebang_python("#!%s\n" % link) == (str(link), [])


SCRIPT = r'''#!%(python)s
import os, sys, time
restart = int(os.environ["TPI_RESTART_COUNT"])
print("incarnation %%d torch-preloaded %%s name %%s argv0 %%s path0 %%s preloaded %%s standby %%s" %% (
    restart, "torch" in sys.modules, __name__, sys.argv[0], sys.path[0],
    os.environ.get("TPI_PRELOADED"), os.environ.get("TPI_STANDBY")), flush=True)
if restart == 0:
    while True:  # preempted: SIGTERM ends it, the supervisor respawns the rank
        time.sleep(0.05)
sys.exit(7 if restart == 1 else 0)
'''


def _wait_event(task, pred, timeout):
    deadline = time.time() + timeout
    while time.time() < deadline:
        for e in task.events():
            if pred(e):
                return e
        time.sleep(0.1)
    raise AssertionError("no such event; events: %s" % [(e.code, e.description)
                                                         for e in task.events()])


def test_a_preempted_rank_resumes_in_its_preloaded_successor(tmp_path):
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(environment=Environment(
        script=SCRIPT % {"python": sys.executable}, timeout=120,
        variables=Variables({"TPI_TASK": "true", "TPI_PRELOAD": "1",
                             "TPI_MAX_RESTARTS": "1"})))
    task = backends.new(cloud, new_deterministic_identifier("preload-1"), spec)
    task.create()
    try:
        started = _wait_event(task, lambda e: e.code == "standby-start" and
                              "preloaded" in e.description, 60)
        assert "restart 1" in started.description
        time.sleep(4.0)  # the successor is importing torch; activated before or after, it waits
        t0 = time.time()
        task.preempt()
        status = task.wait(60)
        took = time.time() - t0
    finally:
        logs = "\n".join(task.logs())
    # the second incarnation exits 7: a failure the status records
    assert status["failed"] == 1, (status, logs)
    assert "incarnation 0 torch-preloaded False name __main__" in logs, logs
    line = next(l for l in logs.splitlines() if "incarnation 1" in l)
    script_path = line.split(" argv0 ")[1].split()[0]
    assert "torch-preloaded True" in line and "name __main__" in line, line
    assert line.split(" path0 ")[1].split()[0] == os.path.dirname(script_path), line
    assert "standby None" in line and "preloaded None" not in line, line
    starts = [e for e in task.events() if e.code == "rank-start"]
    assert any("warm standby" in e.description and "restart 1" in e.description
               for e in starts), starts
    assert took < 30, took
    # the successor's own parked successor was discarded unused: it leaves no empty log
    assert all(l.strip() for l in task.logs()), task.logs()
    task.delete()


def test_preload_is_on_by_default_and_off_on_request(tmp_path, monkeypatch):
    monkeypatch.delenv("TPI_PRELOAD", raising=False)  # tests/conftest.py turns it off
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))

    def argv_for(script, **env):
        spec = Task(environment=Environment(script=script, variables=Variables(env)))
        task = backends.new(cloud, new_deterministic_identifier("pre-%d" % len(env)), spec)
        return task._preload_argv(lambda name, default: env.get(name, default))

    python_script = "#!%s\nprint(1)\n" % sys.executable
    argv = argv_for(python_script)
    assert argv[0] == sys.executable and argv[1] == "-c" and "runtime.preload" in argv[2]
    assert argv_for(python_script, TPI_PRELOAD="0") == []
    assert "gpu=True" in argv_for(python_script, TPI_PRELOAD="gpu")[2]
    assert "gpu='lite'" in argv_for(python_script, TPI_PRELOAD="gpu-lite")[2]
    assert "gpu=False" in argv[2]
    assert argv_for(python_script, TPI_WARM_STANDBY="hot") == []  # its own parked successor
    assert argv_for("#!/bin/sh\necho hi\n") == []


def test_no_preload_when_disabled(tmp_path):
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(environment=Environment(
        script="#!%s\nimport time; time.sleep(3)\n" % sys.executable, timeout=60,
        variables=Variables({"TPI_TASK": "true", "TPI_PRELOAD": "0"})))
    task = backends.new(cloud, new_deterministic_identifier("preload-0"), spec)
    task.create()
    assert task.wait(60)["succeeded"] == 1
    assert not [e for e in task.events() if e.code == "standby-start"]
    task.delete()


GANG = r'''#!%(python)s
import os, sys, time
restart = int(os.environ["TPI_RESTART_COUNT"])
print("rank %%s incarnation %%d torch-preloaded %%s port %%s" %% (
    os.environ["RANK"], restart, "torch" in sys.modules, os.environ["MASTER_PORT"]), flush=True)
if restart == 0:
    while True:
        time.sleep(0.05)
'''


def test_a_preempted_gang_resumes_in_preloaded_successors_on_the_new_port(tmp_path):
    """Two coupled ranks, both preempted: each resumes in its own preloaded successor, which
    takes the new incarnation's rendezvous port from its activation ("go port=N")."""
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(environment=Environment(
        script=GANG % {"python": sys.executable}, timeout=120,
        variables=Variables({"TPI_TASK": "true", "TPI_PRELOAD": "1", "TPI_MAX_RESTARTS": "1"})),
        parallelism=2)
    task = backends.new(cloud, new_deterministic_identifier("preload-gang"), spec)
    task.create()
    try:
        deadline = time.time() + 60
        while time.time() < deadline and len([
                e for e in task.events()
                if e.code == "standby-start" and "preloaded" in e.description]) < 2:
            time.sleep(0.1)
        time.sleep(4.0)
        task.preempt()
        status = task.wait(60)
    finally:
        logs = "\n".join(task.logs())
    assert status["succeeded"] == 2, (status, logs)
    first = {l.split()[2]: l.split()[-1] for l in logs.splitlines() if "incarnation 0" in l}
    second = [l for l in logs.splitlines() if "incarnation 1" in l]
    assert len(first) == 2 and len(second) == 2, logs
    for line in second:
        words = line.split()
        assert "torch-preloaded True" in line, line
        assert words[-1] != first[words[2]], (line, first)  # a fresh rendezvous port
    task.delete()


def test_shell_scripts_that_run_one_python_file_are_preloaded():
    from terraform_provider_iterative_amd.backends.node import shell_python_command

    exe = sys.executable
    assert shell_python_command("#!/bin/bash\nset -e\n%s train.py --lr 1e-4\n" % exe) == \
        (exe, [], ["train.py", "--lr", "1e-4"])
    assert shell_python_command("#!/bin/sh\n# run it\nexec %s -u x.py\n" % exe) is None  # -u
    for script in ("#!/bin/bash\npip install -r r.txt\n%s train.py\n" % exe,  # two commands
                   "#!/bin/bash\n%s train.py > log\n" % exe,                   # redirection
                   "#!/bin/bash\n%s train.py $ARGS\n" % exe,                   # expansion
                   "#!/bin/bash\n%s -m pkg.train\n" % exe,                     # a module
                   "#!/bin/bash\n/nonexistent/python3 train.py\n",             # another python
                   "#!/usr/bin/env python3\nprint(1)\n"):                      # not a shell
        assert shell_python_command(script) is None, script


WRAPPED = r'''import os, sys, time
restart = int(os.environ["TPI_RESTART_COUNT"])
print("incarnation %d torch-preloaded %s argv %s" % (restart, "torch" in sys.modules,
                                                     " ".join(sys.argv[1:])), flush=True)
if restart == 0:
    while True:
        time.sleep(0.05)
'''


def test_a_shell_wrapped_python_rank_resumes_in_a_preloaded_successor(tmp_path):
    work = tmp_path / "work"
    work.mkdir()
    (work / "train.py").write_text(WRAPPED)
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(environment=Environment(
        script="#!/bin/bash\nset -e\nexec %s train.py --epochs 3\n" % sys.executable,
        timeout=120, directory=str(work),
        variables=Variables({"TPI_TASK": "true", "TPI_PRELOAD": "1", "TPI_MAX_RESTARTS": "1"})))
    task = backends.new(cloud, new_deterministic_identifier("preload-sh"), spec)
    task.create()
    try:
        _wait_event(task, lambda e: e.code == "standby-start" and "preloaded" in e.description,
                    60)
        time.sleep(4.0)
        task.preempt()
        status = task.wait(60)
    finally:
        logs = "\n".join(task.logs())
    assert status["succeeded"] == 1, (status, logs)
    assert "incarnation 0 torch-preloaded False argv --epochs 3" in logs, logs
    assert "incarnation 1 torch-preloaded True argv --epochs 3" in logs, logs
    task.delete()


def test_an_unused_preloaded_successor_leaves_no_log(tmp_path):
    """The rank finishes normally: its parked successor is discarded without having run, and
    `leo read` shows the rank's log only (no empty machine log)."""
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(environment=Environment(
        script="#!%s\nimport time\nprint('working', flush=True)\ntime.sleep(5)\n" % sys.executable,
        timeout=60, variables=Variables({"TPI_TASK": "true", "TPI_PRELOAD": "1"})))
    task = backends.new(cloud, new_deterministic_identifier("preload-unused"), spec)
    task.create()
    assert task.wait(60)["succeeded"] == 1
    codes = [e.code for e in task.events()]
    assert "standby-start" in codes and "standby-discarded" in codes, codes
    logs = task.logs()
    assert len(logs) == 1 and "working" in logs[0], logs
    task.delete()


EVIDENCE = r'''#!%(python)s
import os, sys, time
restart = int(os.environ["TPI_RESTART_COUNT"])
if restart == 0:
    dev = open(%(device)r, "rb")  # "initialises the GPU": the main process holds the device
    if %(fork)r and os.fork() == 0:  # a worker forked after that holds it too
        while True:
            time.sleep(0.05)
    print("incarnation 0 holds the device", flush=True)
    while True:
        time.sleep(0.05)
print("incarnation %%d warmed %%s" %% (restart, os.environ.get("TPI_PRELOAD_GPU_WARMED")),
      flush=True)
'''


def _evidence_task(tmp_path, fork, name):
    device = tmp_path / "fake-kfd"
    device.write_bytes(b"")
    cloud = Cloud(provider="local",
                  credentials=Credentials(node=NodeCredentials(state_root=str(tmp_path / "st"))))
    spec = Task(environment=Environment(
        script=EVIDENCE % {"python": sys.executable, "device": str(device), "fork": fork},
        timeout=120, variables=Variables({"TPI_TASK": "true", "TPI_PRELOAD": "1",
                                          "TPI_MAX_RESTARTS": "1",
                                          "TPI_PRELOAD_GPU_DEVICE": str(device)})))
    return backends.new(cloud, new_deterministic_identifier(name), spec)


def test_the_preloaded_successor_warms_its_gpu_on_evidence(tmp_path):
    """the default cold successor gets its GPU context before the preemption
    when the running rank shows it is safe -- its main process alone holds the GPU device
    (faked here by a file, ``TPI_PRELOAD_GPU_DEVICE``) -- and the activation names it."""
    task = _evidence_task(tmp_path, False, "preload-evidence")
    task.create()
    try:
        warm = _wait_event(task, lambda e: e.code == "preload-gpu-warm", 60)
        assert "alone holds" in " ".join(warm.description)
        time.sleep(2.0)  # the parked successor finishes importing (and tries its warm-up)
        task.preempt()
        status = task.wait(60)
    finally:
        logs = "\n".join(task.logs())
    assert status["succeeded"] == 1, (status, logs)
    line = next(l for l in logs.splitlines() if "incarnation 1" in l)
    assert "warmed None" not in line, line  # the successor did run its warm-up (no GPU: -1)
    starts = [e for e in task.events() if e.code == "rank-start" and "restart 1" in e.description]
    assert starts and "GPU warmed" in starts[0].description, starts
    assert not any(e.code == "preload-plain" for e in task.events())
    task.delete()


def test_a_script_whose_workers_hold_the_gpu_keeps_a_plain_successor(tmp_path):
    """A script with other processes on the GPU (forked workers, or a fork after the GPU was
    initialised) gets a plain preloaded successor: no context inherited by what it forks."""
    task = _evidence_task(tmp_path, True, "preload-plain")
    task.create()
    try:
        plain = _wait_event(task, lambda e: e.code == "preload-plain", 60)
        assert "2 processes of the rank hold" in " ".join(plain.description)
        time.sleep(1.5)
        assert not any(e.code == "preload-gpu-warm" for e in task.events())
        task.preempt()
        status = task.wait(60)
    finally:
        logs = "\n".join(task.logs())
    assert status["succeeded"] == 1, (status, logs)
    line = next(l for l in logs.splitlines() if "incarnation 1" in l)
    assert "warmed None" in line, line
    starts = [e for e in task.events() if e.code == "rank-start" and "restart 1" in e.description]
    assert starts and "preloaded" in starts[0].description and \
        "GPU warmed" not in starts[0].description, starts
    task.delete()
