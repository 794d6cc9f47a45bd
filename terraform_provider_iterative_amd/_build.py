"""In-tree build of the native components (no setuptools, no JIT cache).

* ``_lib/_tpi_native*.so``  host C++ (pybind11): filters, walker/transfer, CRC32C, XXH64,
  CPU pack/unpack.
* ``_lib/libtpi_hip.so``    HIP/CDNA4 kernels + checkpoint engine, ``--offload-arch=gfx950``,
  linked against the libamdhip64 that ships with torch so one HIP runtime is loaded.
* ``_lib/tpi-supervisor``   the on-node rank supervisor (C++ executable).

Rebuilds are incremental on source mtimes.  ``python -m terraform_provider_iterative_amd._build``
builds everything; ``__graft_entry__.build()`` calls :func:`build_all`.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List, Sequence

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
LIB = os.path.join(PKG, "_lib")
ROCM_LIB = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"

NATIVE_SO = os.path.join(LIB, "_tpi_native" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
HIP_SO = os.path.join(LIB, "libtpi_hip.so")
SUPERVISOR = os.path.join(LIB, "tpi-supervisor")


def _sources(*patterns: str) -> List[str]:
    out: List[str] = []
    for pattern in patterns:
        out.extend(sorted(glob.glob(os.path.join(CSRC, pattern))))
    return out


def _stale(target: str, deps: Sequence[str]) -> bool:
    if not os.path.exists(target):
        return True
    mtime = os.path.getmtime(target)
    return any(os.path.getmtime(dep) > mtime for dep in deps)


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    result = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if result.returncode != 0:
        raise RuntimeError("build failed: %s\n%s" % (" ".join(cmd), result.stdout))


def _atomic_output(target: str) -> str:
    os.makedirs(os.path.dirname(target), exist_ok=True)
    return target + ".tmp.%d" % os.getpid()


def build_native(force: bool = False, verbose: bool = False) -> str:
    srcs = _sources("native/*.cpp")
    deps = srcs + _sources("native/*.h", "common/*.h", "hip/tpi_hip.h")
    if force or _stale(NATIVE_SO, deps):
        import pybind11

        tmp = _atomic_output(NATIVE_SO)
        cxx = os.environ.get("CXX", "g++")
        _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-msse4.2", "-pthread",
              "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
              "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"],
              *srcs, "-o", tmp], verbose)
        os.replace(tmp, NATIVE_SO)
    return NATIVE_SO


def torch_lib_dir() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        raise RuntimeError("torch is required to link libtpi_hip.so")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def build_hip(force: bool = False, verbose: bool = False) -> str:
    srcs = _sources("hip/*.hip")
    deps = srcs + _sources("hip/*.h", "common/*.h")
    if force or _stale(HIP_SO, deps):
        tl = torch_lib_dir()
        tmp = _atomic_output(HIP_SO)
        _run([hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
              "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics",
              *srcs, "-L" + tl, "-Wl,-rpath," + tl, "-L" + ROCM_LIB, "-Wl,-rpath," + ROCM_LIB,
              "-lrocprofiler-sdk-roctx", "-o", tmp], verbose)
        os.replace(tmp, HIP_SO)
    return HIP_SO


def build_supervisor(force: bool = False, verbose: bool = False) -> str:
    srcs = _sources("supervisor/*.cpp")
    if not srcs:
        return ""
    deps = srcs + _sources("supervisor/*.h")
    if force or _stale(SUPERVISOR, deps):
        tmp = _atomic_output(SUPERVISOR)
        cxx = os.environ.get("CXX", "g++")
        _run([cxx, "-O2", "-std=c++17", "-Wall", "-pthread", *srcs, "-o", tmp], verbose)
        os.replace(tmp, SUPERVISOR)
    return SUPERVISOR


def build_all(force: bool = False, verbose: bool = False, hip: bool = True) -> List[str]:
    outs = [build_native(force, verbose), build_supervisor(force, verbose)]
    if hip:
        outs.append(build_hip(force, verbose))
    return [o for o in outs if o]


if __name__ == "__main__":
    for path in build_all(force="--force" in sys.argv, verbose=True,
                          hip="--no-hip" not in sys.argv):
        print(path)
