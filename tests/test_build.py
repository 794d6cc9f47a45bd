"""Build reproducibility and version plumbing (reference: Makefile:10 ``-X utils.Version``)."""
import os
import subprocess
import sys

from terraform_provider_iterative_amd import __version__, _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stamps_track_content_not_mtimes(tmp_path):
    src = tmp_path / "a.cpp"
    src.write_text("int x = 1;\n")
    target = tmp_path / "out.bin"
    target.write_bytes(b"built")
    cmd = ["g++", "-O2", str(src), "-o", "@OUT@"]
    assert _build._stale(str(target), cmd, [str(src)])  # no stamp yet
    _build._stamp(str(target), cmd, [str(src)])
    assert not _build._stale(str(target), cmd, [str(src)])
    os.utime(src, (1, 1))  # a checkout with arbitrary mtimes changes nothing
    assert not _build._stale(str(target), cmd, [str(src)])
    src.write_text("int x = 2;\n")
    assert _build._stale(str(target), cmd, [str(src)])
    _build._stamp(str(target), cmd, [str(src)])
    assert _build._stale(str(target), cmd + ["-g"], [str(src)])  # flags count too


def test_built_artefacts_are_not_tracked():
    out = subprocess.run(["git", "ls-files", "terraform_provider_iterative_amd/_lib"], cwd=ROOT,
                         capture_output=True, text=True)
    assert out.returncode != 0 or out.stdout.strip() == ""


def test_version_everywhere():
    env = dict(os.environ, PYTHONPATH=ROOT)
    for argv, expect in ((["bin/leo", "--version"], "leo version " + __version__),
                         (["bin/tpi", "version"], "tpi v" + __version__),
                         (["bin/tpi", "-version"], "tpi v" + __version__),
                         (["bin/terraform-provider-iterative", "--version"], "v" + __version__)):
        res = subprocess.run([sys.executable] + argv, cwd=ROOT, env=env, capture_output=True,
                             text=True, timeout=60)
        assert res.returncode == 0 and expect in res.stdout, (argv, res.stdout, res.stderr)
    sup = subprocess.run([_build.build_supervisor(), "--version"], capture_output=True, text=True)
    assert sup.stdout.strip() == "tpi-supervisor " + __version__
    from terraform_provider_iterative_amd.ops import native

    assert native().VERSION == __version__
    from terraform_provider_iterative_amd.utils import analytics

    assert analytics.VERSION == __version__


def test_stamps_survive_moving_the_tree(tmp_path):
    """A GPU box runs a snapshot of the tree from a scratch directory: the stamps built here
    must still match there, or the first use on every box recompiles (libtpi_hip: minutes)."""
    import shutil

    _build.build_native()
    _build.build_supervisor()
    _build.build_torch_ext()  # depends on a file outside the tree (torch's version.py)
    copy = tmp_path / "elsewhere" / "at" / "another" / "depth"
    shutil.copytree(os.path.join(ROOT, "csrc"), copy / "csrc")
    shutil.copytree(os.path.join(ROOT, "terraform_provider_iterative_amd"),
                    copy / "terraform_provider_iterative_amd",
                    ignore=shutil.ignore_patterns("__pycache__"))
    code = ("from terraform_provider_iterative_amd import _build as b\n"
            "import pybind11, sysconfig\n"
            "assert b.ROOT == %r, b.ROOT\n"
            "srcs = b._sources('supervisor/*.cpp')\n"
            "cmd = [__import__('os').environ.get('CXX', 'g++'), '-O2', '-std=c++17', '-Wall', "
            "'-pthread', b._define_version(), *srcs, '-o', '@OUT@']\n"
            "assert not b._stale(b.SUPERVISOR, cmd, srcs + b._sources('supervisor/*.h'))\n"
            "import torch  # (build_torch_ext imports it; not part of the timing)\n"
            "import time; t = time.time(); b.build_native(); b.build_supervisor()\n"
            "b.build_torch_ext()\n"
            "assert time.time() - t < 2, 'rebuilt'\n" % str(copy))
    res = subprocess.run([sys.executable, "-c", code], cwd=str(copy), capture_output=True,
                         text=True, timeout=120)
    assert res.returncode == 0, res.stderr


def test_fast_path_skips_the_content_check_only_while_nothing_changed(tmp_path, monkeypatch):
    """``tpi apply`` checks the supervisor's and the native module's stamps before every task
    start: while no dependency's size or mtime moved, the ``.fast`` signature answers without
    reading and hashing the sources; any change goes back to the content check."""
    src = tmp_path / "a.cpp"
    src.write_text("int x = 1;\n")
    target = tmp_path / "out.bin"
    target.write_bytes(b"built")
    cmd = ["g++", "-O2", str(src), "-o", "@OUT@"]
    assert not _build._fast_fresh(str(target), [str(src)])
    _build._stamp(str(target), cmd, [str(src)])  # a build writes both
    assert _build._fast_fresh(str(target), [str(src)])
    os.utime(src, (1, 1))  # a checkout with other mtimes: back to the content check ...
    assert not _build._fast_fresh(str(target), [str(src)])
    assert not _build._stale(str(target), cmd, [str(src)])  # ... which still matches
    _build._write_fast(str(target), [str(src)])
    assert _build._fast_fresh(str(target), [str(src)])
    src.write_text("int x = 22;\n")  # an edit changes size and mtime
    assert not _build._fast_fresh(str(target), [str(src)])
    assert _build._stale(str(target), cmd, [str(src)])
    _build._write_fast(str(target), [str(src)])
    monkeypatch.setenv("CXX", "clang++")  # the compiler is part of the signature
    assert not _build._fast_fresh(str(target), [str(src)])
