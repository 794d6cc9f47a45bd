"""In-tree build of the native components (no setuptools, no JIT cache).

* ``_lib/_tpi_native*.so``  host C++ (pybind11): filters, walker/transfer, CRC32C, XXH64,
  CPU pack/unpack.
* ``_lib/libtpi_hip.so``    HIP/CDNA4 kernels, checkpoint/staging engine and the RCCL task
  communicator, ``--offload-arch=gfx950``.  It needs ``libamdhip64.so.7`` / ``librccl.so.1``
  by soname: in a PyTorch process (``ops._loader`` always imports torch first) those sonames
  are torch's bundled runtime (HIP 7.0), so one HIP runtime is loaded there.
* ``_lib/tpi-supervisor``   the on-node rank supervisor (C++ executable, no HIP).
* ``_lib/tpi-stager``       the per-task workdir stager (C++/HIP executable on libtpi_hip).  No
  torch in it: its sonames resolve to /opt/rocm's runtime (HIP 7.2).  Its HBM images are
  therefore exported by 7.2 and imported by the ranks' 7.0 runtime -- the pairing that opens
  allocations of 2 GiB and more (``profiles/round6/ipc_runtime.md``).

Nothing built is tracked by git.  A target is rebuilt when its ``.stamp`` (SHA-256 of the
compile command and of every source/header it depends on) no longer matches -- content, not
mtimes, so a fresh checkout (where every file has the checkout's mtime) always compiles from
source.  The content check costs a few ms (reading and hashing every source, importing
pybind11 for the command), which ``tpi apply`` would pay before every task start; a ``.fast``
file next to the stamp records the size and mtime of every dependency, of the target and of
this file as they were when the content last matched, and while all of them are unchanged the
content check is skipped (any change, a fresh checkout included, goes back to it).  ``python -m terraform_provider_iterative_amd._build`` builds everything;
``__graft_entry__.build()`` calls :func:`build_all`.  The release version
(``_version.py``, the reference's ``-X utils.Version``, ``Makefile:10``) is compiled into every
native component as ``TPI_VERSION_STRING``.
"""
from __future__ import annotations

import glob
import importlib.machinery
import os
import shutil
import subprocess
import sys
from typing import List, Sequence

try:  # the builtin module: hashlib would load OpenSSL on every CLI start (~4 ms)
    from _sha256 import sha256 as _sha256
except ImportError:  # pragma: no cover
    from hashlib import sha256 as _sha256

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
LIB = os.path.join(PKG, "_lib")
ROCM_LIB = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"

# the interpreter's extension suffix (sysconfig's EXT_SUFFIX) without importing sysconfig,
# which costs `tpi apply` ~3 ms per start; sysconfig is imported where a build needs it
_EXT_SUFFIX = importlib.machinery.EXTENSION_SUFFIXES[0]
NATIVE_SO = os.path.join(LIB, "_tpi_native" + _EXT_SUFFIX)
HIP_SO = os.path.join(LIB, "libtpi_hip.so")
SUPERVISOR = os.path.join(LIB, "tpi-supervisor")
STAGER = os.path.join(LIB, "tpi-stager")
TORCH_EXT = os.path.join(LIB, "_tpi_torch" + _EXT_SUFFIX)


def _sources(*patterns: str) -> List[str]:
    out: List[str] = []
    for pattern in patterns:
        out.extend(sorted(glob.glob(os.path.join(CSRC, pattern))))
    return out


def version() -> str:
    from ._version import __version__

    return os.environ.get("TPI_VERSION", __version__)


def _digest(cmd: Sequence[str], deps: Sequence[str]) -> str:
    # Paths inside the tree are hashed relative to it: a copy of the tree elsewhere (a GPU
    # box runs a snapshot from a scratch directory) keeps its stamps valid instead of
    # recompiling everything on first use.
    h = _sha256()
    h.update("\0".join(c.replace(ROOT, "@ROOT@") for c in cmd if ".tmp." not in c).encode())
    for dep in sorted(set(deps)):
        # outside the tree (torch's version file): the absolute path, the same on every box
        name = os.path.relpath(dep, ROOT) if dep.startswith(ROOT + os.sep) else dep
        h.update(b"\0" + name.encode() + b"\0")
        with open(dep, "rb") as handle:
            h.update(handle.read())
    return h.hexdigest()


def _stale(target: str, cmd: Sequence[str], deps: Sequence[str]) -> bool:
    """True unless ``target`` exists and its stamp matches the command + dependency content."""
    if not os.path.exists(target):
        return True
    try:
        with open(target + ".stamp") as handle:
            return handle.read().strip() != _digest(cmd, deps)
    except OSError:
        return True


def _stamp(target: str, cmd: Sequence[str], deps: Sequence[str]) -> None:
    with open(target + ".stamp", "w") as handle:
        handle.write(_digest(cmd, deps) + "\n")
    _write_fast(target, deps)


_FAST_ENV = ("CXX", "ROCM_PATH", "PYTORCH_ROCM_ARCH", "TPI_VERSION")


def _fast_signature(target: str, deps: Sequence[str]) -> str:
    """Sizes and mtimes of ``target``, its dependencies and this file, plus the environment
    the command depends on (its compiler, ROCm, architecture, version)."""
    parts = ["%s=%s" % (k, os.environ.get(k, "")) for k in _FAST_ENV]
    for path in [target, os.path.abspath(__file__), *sorted(set(deps))]:
        st = os.stat(path)
        name = os.path.relpath(path, ROOT) if path.startswith(ROOT + os.sep) else path
        parts.append("%s:%d:%d" % (name, st.st_size, st.st_mtime_ns))
    return "\n".join(parts)


def _fast_fresh(target: str, deps: Sequence[str]) -> bool:
    """True when nothing :func:`_fast_signature` covers changed since the content last matched."""
    try:
        with open(target + ".fast") as handle:
            return handle.read() == _fast_signature(target, deps)
    except OSError:
        return False


def _write_fast(target: str, deps: Sequence[str]) -> None:
    try:
        tmp = target + ".fast.tmp.%d" % os.getpid()
        with open(tmp, "w") as handle:
            handle.write(_fast_signature(target, deps))
        os.replace(tmp, target + ".fast")
    except OSError:
        pass


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    result = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if result.returncode != 0:
        raise RuntimeError("build failed: %s\n%s" % (" ".join(cmd), result.stdout))


def _atomic_output(target: str) -> str:
    os.makedirs(os.path.dirname(target), exist_ok=True)
    return target + ".tmp.%d" % os.getpid()


def _build(target: str, cmd: List[str], deps: Sequence[str], force: bool,
           verbose: bool) -> str:
    """Compile ``cmd`` (whose output is the placeholder ``@OUT@``) into ``target`` when stale."""
    if not force and not _stale(target, cmd, deps):
        _write_fast(target, deps)  # the content matched: skip the hashing next time
        return target
    tmp = _atomic_output(target)
    _run([tmp if c == "@OUT@" else c for c in cmd], verbose)
    os.replace(tmp, target)
    _stamp(target, cmd, deps)
    return target


def _define_version() -> str:
    return '-DTPI_VERSION_STRING="%s"' % version()


def build_native(force: bool = False, verbose: bool = False) -> str:
    srcs = _sources("native/*.cpp")
    deps = srcs + _sources("native/*.h", "common/*.h", "hip/tpi_hip.h")
    if not force and _fast_fresh(NATIVE_SO, deps):
        return NATIVE_SO
    import sysconfig

    import pybind11

    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-msse4.2", "-pthread",
           "-fvisibility=hidden", "-Wall", "-Wno-unused-function", _define_version(),
           "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"],
           *srcs, "-o", "@OUT@"]
    return _build(NATIVE_SO, cmd, deps, force, verbose)


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
    """``libtpi_hip.so``: every source compiled to its own object in parallel (each carries
    its own gfx950 code object; the kernels are reached through host launch functions, so no
    relocatable device code is needed), then one link."""
    srcs = _sources("hip/*.hip", "hip/*.cpp")
    headers = _sources("hip/*.h", "common/*.h")
    tl = torch_lib_dir()
    flags = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-Wno-unused-function", "-munsafe-fp-atomics", _define_version()]
    objdir = os.path.join(LIB, "obj")
    os.makedirs(objdir, exist_ok=True)

    def compile_one(src: str) -> str:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        return _build(obj, [hipcc(), *flags, "-c", src, "-o", "@OUT@"], [src] + headers,
                      force, verbose)

    from concurrent.futures import ThreadPoolExecutor

    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", "0") or os.cpu_count() or 4)))
    with ThreadPoolExecutor(jobs) as pool:
        objs = list(pool.map(compile_one, srcs))
    cmd = [hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", *objs, "-L" + tl,
           "-Wl,-rpath," + tl, "-L" + ROCM_LIB, "-Wl,-rpath," + ROCM_LIB, "-lrccl",
           "-lrocprofiler-sdk-roctx", "-ldl", "-o", "@OUT@"]
    return _build(HIP_SO, cmd, objs, force, verbose)


def build_supervisor(force: bool = False, verbose: bool = False) -> str:
    srcs = _sources("supervisor/*.cpp")
    if not srcs:
        return ""
    deps = srcs + _sources("supervisor/*.h")
    if not force and _fast_fresh(SUPERVISOR, deps):
        return SUPERVISOR
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O2", "-std=c++17", "-Wall", "-pthread", _define_version(), *srcs,
           "-o", "@OUT@"]
    return _build(SUPERVISOR, cmd, deps, force, verbose)


def build_stager(force: bool = False, verbose: bool = False) -> str:
    """The per-task workdir stager (links libtpi_hip.so next to it; no Python, no torch)."""
    srcs = _sources("stager/*.cpp")
    if not srcs:
        return ""
    hip_so = build_hip(force, verbose)
    deps = srcs + [hip_so] + _sources("hip/tpi_hip.h", "common/*.h", "supervisor/json.h")
    tl = torch_lib_dir()
    cmd = [hipcc(), "-O2", "-std=c++17", "-Wall", "-pthread", _define_version(), *srcs,
           "-L" + LIB, "-ltpi_hip", "-Wl,-rpath,$ORIGIN", "-L" + tl, "-Wl,-rpath," + tl,
           "-L" + ROCM_LIB, "-Wl,-rpath," + ROCM_LIB, "-o", "@OUT@"]
    return _build(STAGER, cmd, deps, force, verbose)


def build_torch_ext(force: bool = False, verbose: bool = False) -> str:
    """``_tpi_torch``: torch helpers that release the GIL (``csrc/torchext``; host code against
    torch's own headers and libraries, same C++ ABI)."""
    srcs = _sources("torchext/*.cpp")
    if not srcs:
        return ""
    import torch

    import sysconfig

    inc = os.path.join(os.path.dirname(torch.__file__), "include")
    tl = torch_lib_dir()
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-D_GLIBCXX_USE_CXX11_ABI=%d" % int(torch._C._GLIBCXX_USE_CXX11_ABI),
           "-DTORCH_EXTENSION_NAME=_tpi_torch", "-DTORCH_API_INCLUDE_EXTENSION_H",
           "-isystem", inc, "-isystem", os.path.join(inc, "torch", "csrc", "api", "include"),
           "-isystem", sysconfig.get_paths()["include"], *srcs, "-L" + tl, "-Wl,-rpath," + tl,
           "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-o", "@OUT@"]
    # torch's version file is a dependency: a different torch needs a rebuild
    deps = srcs + [os.path.join(os.path.dirname(torch.__file__), "version.py")]
    return _build(TORCH_EXT, cmd, deps, force, verbose)


def build_all(force: bool = False, verbose: bool = False, hip: bool = True) -> List[str]:
    outs = [build_native(force, verbose), build_supervisor(force, verbose),
            build_torch_ext(force, verbose)]
    if hip:
        outs.append(build_hip(force, verbose))
        outs.append(build_stager(force, verbose))
    return [o for o in outs if o]


if __name__ == "__main__":
    for path in build_all(force="--force" in sys.argv, verbose=True,
                          hip="--no-hip" not in sys.argv):
        print(path)
