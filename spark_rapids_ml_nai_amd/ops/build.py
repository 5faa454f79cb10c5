"""Build ``libsrml_ops.so`` (all HIP kernels, gfx950) in-tree with hipcc.

Every ``csrc/*.hip`` translation unit is compiled to an object in parallel and linked into
one shared library under ``ops/lib/``. The library is loaded with ctypes (``ops/native.py``)
into the same process as PyTorch-ROCm; it links ``libamdhip64.so.7``, which resolves to the
HIP runtime torch already loaded, so kernels launch on torch's current HIP stream.

Usage: ``python -m spark_rapids_ml_nai_amd.ops.build [--force]``
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
from typing import List

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(HERE, "lib", "obj")
LIBNAME = "libsrml_ops.so"
ARCH = os.environ.get("SRML_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found; install ROCm or set HIPCC")


def lib_path() -> str:
    return os.path.join(LIBDIR, LIBNAME)


def _sources() -> List[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _headers() -> List[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.h")))


def _flags() -> List[str]:
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-ffp-contract=fast",
            "-munsafe-fp-atomics"]


def needs_build() -> bool:
    out = lib_path()
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in _sources() + _headers() + [__file__])


def _compile(src: str) -> str:
    obj = os.path.join(OBJDIR, os.path.basename(src).replace(".hip", ".o"))
    hdr_t = max([os.path.getmtime(h) for h in _headers()] + [0])
    if os.path.exists(obj) and os.path.getmtime(obj) > max(os.path.getmtime(src), hdr_t, os.path.getmtime(__file__)):
        return obj
    cmd = [hipcc()] + _flags() + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, " ".join(cmd), r.stderr[-8000:]))
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    if not force and not needs_build():
        return lib_path()
    if force:
        for o in glob.glob(os.path.join(OBJDIR, "*.o")):
            os.remove(o)
    srcs = _sources()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(_compile, srcs))
    tmp = lib_path() + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s" % r.stderr[-8000:])
    os.replace(tmp, lib_path())
    if verbose:
        print("built", lib_path())
    return lib_path()


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
