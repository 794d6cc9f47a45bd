"""Machine-script renderer: golden outputs (minimal/full, like script_test.go) and an actual
run of the rendered bootstrap against the native supervisor."""
import json
import os
import subprocess
import time


from terraform_provider_iterative_amd import _build
from terraform_provider_iterative_amd.models.values import Variables
from terraform_provider_iterative_amd.runtime.machine_script import render

GOLDEN = os.path.join(os.path.dirname(__file__), "testdata")
SCRIPT = "#!/bin/sh\necho \"done\"\n"


def _golden(name, text):
    path = os.path.join(GOLDEN, name)
    if os.environ.get("UPDATE_GOLDEN") or not os.path.exists(path):
        os.makedirs(GOLDEN, exist_ok=True)
        with open(path, "w") as f:
            f.write(text)
    with open(path) as f:
        assert f.read() == text


def test_golden_minimal():
    _golden("machine_script_minimal.golden", render(SCRIPT))


def test_golden_full():
    out = render(SCRIPT, credentials={"SECRET": "VALUE"}, variables=Variables({"KEY": "VALUE"}),
                 timeout=1659919333, task_id="tpi-test-3z4xlzwq-3u0vweb4", parallelism=2,
                 gpus="0,1", supervisor="/opt/tpi/tpi-supervisor")
    _golden("machine_script_full.golden", out)
    assert "TPI_DEADLINE=1659919333" in out


def test_bootstrap_runs_task(tmp_path):
    supervisor = _build.build_supervisor()
    out = render("#!/bin/sh\necho \"hello $KEY $SECRET\"\n", credentials={"SECRET": "s3 cr'et"},
                 variables=Variables({"KEY": 'quoted "value"'}), task_id="tpi-boot",
                 supervisor=supervisor)
    env = dict(os.environ, TPI_TASK_DIRECTORY=str(tmp_path / "task"))
    env["XDG_RUNTIME_DIR"] = "/nonexistent"  # force the detached path (no user systemd)
    r = subprocess.run(["bash", "-c", out], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    reports = tmp_path / "task" / "reports"
    deadline = time.time() + 20
    while time.time() < deadline:
        logs = [p for p in reports.iterdir() if p.name.startswith("task-")] if reports.exists() else []
        statuses = [p for p in reports.iterdir() if p.name.startswith("status-")] if reports.exists() else []
        if statuses:
            break
        time.sleep(0.05)
    assert logs and 'hello quoted "value" s3 cr\'et' in logs[0].read_text()
    assert json.loads(statuses[0].read_text())["code"] == "0"
    assert oct((tmp_path / "task" / "supervisor" / "credentials").stat().st_mode & 0o777) == "0o600"


def test_past_deadline_does_not_start(tmp_path):
    out = render(SCRIPT, timeout=1000, supervisor="/bin/false")
    env = dict(os.environ, TPI_TASK_DIRECTORY=str(tmp_path / "t"))
    r = subprocess.run(["bash", "-c", out], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "deadline passed" in r.stderr
