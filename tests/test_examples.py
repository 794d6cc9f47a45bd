"""The shipped examples run as documented (examples/hello on CPU, examples/train on GPU)."""
import os
import shutil
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TPI = [sys.executable, os.path.join(ROOT, "bin", "tpi")]


def _tpi(args, cwd, env, timeout=300):
    res = subprocess.run(TPI + args, cwd=cwd, env=env, capture_output=True, text=True,
                         timeout=timeout)
    assert res.returncode == 0, res.stdout + res.stderr
    return res.stdout


def _run_example(name, tmp_path, wait_for, timeout=120):
    work = tmp_path / name
    shutil.copytree(os.path.join(ROOT, "examples", name), work)
    main = work / "main.tf"
    main.write_text(main.read_text().replace('abspath("../..")', '"%s"' % ROOT))
    env = dict(os.environ, TPI_STATE_ROOT=str(tmp_path / "state"))
    _tpi(["init"], str(work), env)
    _tpi(["apply", "-auto-approve"], str(work), env)
    deadline = time.time() + timeout
    logs = ""
    try:
        while time.time() < deadline:
            _tpi(["refresh"], str(work), env)
            logs = _tpi(["output", "logs"], str(work), env)
            if wait_for in logs:
                break
            time.sleep(0.5)
    finally:
        _tpi(["destroy", "-auto-approve"], str(work), env)
    assert wait_for in logs, logs
    return work, logs


def test_hello_example(tmp_path):
    work, logs = _run_example("hello", tmp_path, "hello from")
    assert (work / "results" / "hello.txt").read_text().startswith("hello from")


@pytest.mark.gpu
def test_train_example(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    _, logs = _run_example("train", tmp_path, "done {", timeout=300)
    assert "staged" in logs and "fresh start" in logs
