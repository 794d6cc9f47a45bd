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
