"""Builds the framework's native libraries in-tree.

* ``liboryx_runtime.so`` -- host C++ runtime (append-only log transport, offset store,
  CSV ingest parser, ID dictionary); compiled with ``g++``.
* ``liboryx_kernels.so`` -- hand-written CDNA4 HIP kernels for gfx950 (ALS Gramian/Cholesky
  solve, top-N scoring, k-means assign/accumulate, RDF histograms and tree traversal);
  compiled with ``hipcc --offload-arch=gfx950``.

Both expose a plain C ABI consumed through :mod:`ctypes` (kernels take raw device pointers
and a ``hipStream_t`` from PyTorch), so there is no dependency on torch's C++ headers and a
rebuild takes seconds.  Outputs land in ``oryx_amd/_native/`` and travel with the source tree.
Rebuilds are incremental on source mtimes.
"""

from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_native")

RUNTIME_SO = os.path.join(OUT, "liboryx_runtime.so")
KERNELS_SO = os.path.join(OUT, "liboryx_kernels.so")
TUNING_SO = os.path.join(OUT, "liboryx_kernels_tuning.so")

ARCH = os.environ.get("ORYX_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build HIP kernels)")


def _stale(out: str, sources: List[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n$ %s\n%s" % (" ".join(cmd), r.stdout))


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    os.makedirs(OUT, exist_ok=True)
    if force or _stale(RUNTIME_SO, srcs + hdrs):
        tmp = RUNTIME_SO + ".tmp"
        cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-pthread",
               "-o", tmp] + srcs + ["-lz", "-lssl", "-lcrypto"]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        os.replace(tmp, RUNTIME_SO)
    return RUNTIME_SO


def build_kernels(force: bool = False, verbose: bool = False, tuning: bool = False) -> str:
    """``liboryx_kernels.so``; ``tuning``: ``liboryx_kernels_tuning.so``, the same kernels plus
    the superseded ones of ``csrc/kernels/tuning/`` (A/B runs: ``ORYX_KERNELS_SO`` points at
    it and ``ORYX_ALS_VARIANT`` / ``ORYX_ALS_WIDE_VARIANT`` select them)."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    so = KERNELS_SO
    if tuning:
        srcs += sorted(glob.glob(os.path.join(CSRC, "kernels", "tuning", "*.hip")))
        so = TUNING_SO
    os.makedirs(OUT, exist_ok=True)
    if force or _stale(so, srcs + hdrs):
        hipcc = _hipcc()
        objdir = os.path.join(OUT, "obj")
        os.makedirs(objdir, exist_ok=True)
        objs = []
        # compile translation units in parallel (each is independent)
        procs = []
        for s in srcs:
            o = os.path.join(objdir, os.path.basename(s) + ".o")
            objs.append(o)
            if force or _stale(o, [s] + hdrs):
                cmd = [hipcc, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC",
                       "-munsafe-fp-atomics", "-I", os.path.join(CSRC, "kernels"),
                       "-c", s, "-o", o]
                if verbose:
                    print(" ".join(cmd), flush=True)
                procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE,
                                                    stderr=subprocess.STDOUT, text=True)))
        for cmd, p in procs:
            out, _ = p.communicate()
            if p.returncode != 0:
                raise RuntimeError("native build failed:\n$ %s\n%s" % (" ".join(cmd), out))
        tmp = so + ".tmp"
        cmd = [hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        _check_no_missing_stubs(tmp)
        os.replace(tmp, so)
    return so


def _check_no_missing_stubs(so: str) -> None:
    """A kernel template whose host-side instantiation hipcc silently dropped links into a
    library with an undefined internal symbol that only fails at dlopen on the GPU box;
    catch it here instead."""
    try:
        out = subprocess.run(["nm", "-u", so], capture_output=True, text=True, timeout=60).stdout
    except (OSError, subprocess.SubprocessError):
        return
    missing = [ln.split()[-1] for ln in out.splitlines() if "_GLOBAL__N_" in ln]
    if missing:
        os.unlink(so)
        raise RuntimeError("native build: undefined internal kernel symbols (host stubs not "
                           "emitted): %s" % ", ".join(missing[:4]))


def build(force: bool = False, verbose: bool = False) -> List[str]:
    return [build_runtime(force, verbose), build_kernels(force, verbose)]


if __name__ == "__main__":
    if "--tuning" in sys.argv:
        print(build_kernels(force="--force" in sys.argv, verbose=True, tuning=True))
    else:
        print("\n".join(build(force="--force" in sys.argv, verbose=True)))
