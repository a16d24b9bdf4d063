"""Build libeks_hip.so for gfx950 in-tree (eks_amd/lib/).

    python -m eks_amd.build          # incremental
    python -m eks_amd.build --force  # rebuild everything

Each ``csrc/*.hip`` translation unit is compiled by ``hipcc
--offload-arch=gfx950`` (cross-compiles without a GPU), each host-only
``csrc/*.cpp`` unit by g++, into an object file,
then all objects are linked into one shared library with a plain C ABI
(include/eks_hip.h).  The library is what the Python package binds with
ctypes; it is built in the tree so that it travels with the repository
snapshot to the GPU box.

A second library, ``libeks_torch.so``, registers the same entry points as
PyTorch operators in C++ (``csrc/torch_ops.cpp``: TORCH_LIBRARY(eks, ...),
CUDA-key and Meta kernels); it is compiled against the installed torch's
headers and links libeks_hip.so (``eks_amd.ops`` loads it).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIBNAME = "libeks_hip.so"
TORCH_LIBNAME = "libeks_torch.so"
TORCH_SRC = "torch_ops.cpp"
ARCH = os.environ.get("EKS_OFFLOAD_ARCH", "gfx950")
# The kernels are written for gfx950's 160 KB of LDS per CU (eks_fit.hip's
# selection kernels stage up to ~161 KB; two_pass.hpp sizes its blocks for it):
# another target would fail to compile or mis-size its blocks, so build()
# refuses it with this message.
ARCH_ERROR = (f"eks_amd is written for MI355X (gfx950) only (160 KB of LDS per CU); "
              f"EKS_OFFLOAD_ARCH={ARCH!r} is not supported")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
# EKS_EXTRA_CFLAGS: tuning experiments only (e.g. "-DEKS_K3_D=2"), not used by default
EXTRA = os.environ.get("EKS_EXTRA_CFLAGS", "").split()
# --offload-compress: the gfx950 code objects are stored compressed in the
# fat binary (the HIP runtime inflates them at load): the library shrinks
# ~2.6x (the compiled shapes' member-count / input-type instantiations)
CFLAGS = [*EXTRA, "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "--offload-compress",
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-but-set-variable"]


def lib_path() -> str:
    return os.path.join(LIBDIR, LIBNAME)


def torch_lib_path() -> str:
    return os.path.join(LIBDIR, TORCH_LIBNAME)


def _torch_flags():
    """Compile / link flags of a host-only C++ unit against the installed
    PyTorch-ROCm (what torch.utils.cpp_extension would pass)."""
    import torch
    from torch.utils import cpp_extension
    tdir = os.path.dirname(torch.__file__)
    inc = [f"-I{p}" for p in cpp_extension.include_paths()] + ["-I/opt/rocm/include"]
    abi = int(bool(torch._C._GLIBCXX_USE_CXX11_ABI))
    cflags = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              *inc]
    ldflags = [f"-L{os.path.join(tdir, 'lib')}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
               "-ltorch_hip", "-lamdhip64", f"-L{LIBDIR}", "-leks_hip", "-Wl,-rpath,$ORIGIN"]
    return cflags, ldflags


def build_torch_ops(force: bool = False, verbose: bool = True) -> str:
    """libeks_torch.so: torch.ops.eks.* registered in C++ (csrc/torch_ops.cpp)."""
    src = os.path.join(CSRC, TORCH_SRC)
    out = torch_lib_path()
    if not force and not _stale(out, [src, lib_path(), *glob.glob(os.path.join(REPO, "include", "*.h"))]):
        return out
    cflags, ldflags = _torch_flags()
    cmd = [CXX, *cflags, "-shared", src, "-o", out + ".tmp", *ldflags]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"torch ops build failed:\n{res.stderr[-6000:]}")
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"[eks_amd.build] linked {out}")
    return out


def _deps() -> list[str]:
    # (this file too: its flags are part of every object)
    return sorted(glob.glob(os.path.join(CSRC, "*.hpp")) +
                  glob.glob(os.path.join(REPO, "include", "*.h"))) + [os.path.abspath(__file__)]


def _stale(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


CXX = shutil.which("g++") or "g++"
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall"]


def _compile(src: str, obj: str) -> None:
    if src.endswith(".cpp"):  # host-only units (CSV I/O)
        cmd = [CXX, *CXXFLAGS, "-c", src, "-o", obj]
    else:
        cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src}:\n{res.stderr[-6000:]}")


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> str:
    if ARCH != "gfx950":
        raise RuntimeError(ARCH_ERROR)
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) +
                  [c for c in glob.glob(os.path.join(CSRC, "*.cpp")) if not c.endswith(TORCH_SRC)])
    deps = _deps()
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(OBJDIR, os.path.splitext(os.path.basename(s))[0] + ".o")
        objs.append(o)
        if force or _stale(o, [s, *deps]):
            todo.append((s, o))
    if todo:
        jobs = jobs or min(len(todo), max(1, (os.cpu_count() or 2) // 2), 8)
        if verbose:
            print(f"[eks_amd.build] compiling {len(todo)} unit(s) for {ARCH} with {jobs} job(s)")
        with cf.ThreadPoolExecutor(jobs) as ex:
            for fut in [ex.submit(_compile, s, o) for s, o in todo]:
                fut.result()
    lib = lib_path()
    if todo or _stale(lib, objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-pthread", "-o", lib + ".tmp"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{res.stderr[-4000:]}")
        os.replace(lib + ".tmp", lib)
        if verbose:
            print(f"[eks_amd.build] linked {lib}")
    # the torch operators are an optional second library: a failure there
    # (torch headers missing, an ABI mismatch) must not take the C-ABI library,
    # which the ctypes path and the CLI use, down with it
    try:
        build_torch_ops(force=force, verbose=verbose)
    except Exception as e:  # noqa: BLE001
        print(f"[eks_amd.build] WARNING: torch operators not built ({type(e).__name__}: "
              f"{str(e)[-2000:]}); libeks_hip.so is unaffected", file=sys.stderr)
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs)
    sys.exit(0)
