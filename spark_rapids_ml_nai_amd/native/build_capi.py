"""Build the C-ABI test program (and the JNI shim when a JDK is present) against libsrml_ops.so.

``python -m spark_rapids_ml_nai_amd.native.build_capi [--test]``: compiles
``native/tests/capi_test.cpp`` with hipcc (host code only, links the in-tree library) and, with
``--test``, runs it (needs a GPU).
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys

from ..ops import build as _ops_build

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NATIVE = os.path.join(ROOT, "native")
OUT = os.path.join(os.path.dirname(_ops_build.lib_path()))


def _hipcc() -> str:
    return os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


def build(verbose: bool = False) -> str:
    lib = _ops_build.build()
    libdir = os.path.dirname(lib)
    exe = os.path.join(OUT, "srml_capi_test")
    src = os.path.join(NATIVE, "tests", "capi_test.cpp")
    if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(src), os.path.getmtime(lib)):
        cmd = [_hipcc(), "-O2", "-std=c++17", "-I", os.path.join(NATIVE, "include"), src, "-L", libdir,
               "-l:" + os.path.basename(lib), "-Wl,-rpath," + libdir, "-o", exe]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    # the JNI shim compiled against the test JNIEnv (native/tests/jni_harness) and driven by a
    # C++ harness: runs every JniSRML entry point without a JVM (tests/test_native_capi.py)
    shim = os.path.join(OUT, "srml_jni_shim_test")
    shim_src = [os.path.join(NATIVE, "tests", "jni_shim_test.cpp"), os.path.join(NATIVE, "jni", "srml_jni.cpp")]
    if not os.path.exists(shim) or os.path.getmtime(shim) < max([os.path.getmtime(f) for f in shim_src] +
                                                                [os.path.getmtime(lib)]):
        cmd = [_hipcc(), "-O2", "-std=c++17", "-I", os.path.join(NATIVE, "tests", "jni_harness"), "-I",
               os.path.join(NATIVE, "include")] + shim_src + ["-L", libdir, "-l:" + os.path.basename(lib),
                                                              "-Wl,-rpath," + libdir, "-o", shim]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    jni_inc = _find_jni()
    if jni_inc:
        so = os.path.join(OUT, "libsrml_jni.so")
        cmd = [_hipcc(), "-O2", "-std=c++17", "-shared", "-fPIC", "-I", os.path.join(NATIVE, "include")]
        for d in jni_inc:
            cmd += ["-I", d]
        cmd += [os.path.join(NATIVE, "jni", "srml_jni.cpp"), "-L", libdir, "-l:" + os.path.basename(lib),
                "-Wl,-rpath," + libdir, "-o", so]
        subprocess.check_call(cmd)
    return exe


def shim_test_path() -> str:
    return os.path.join(OUT, "srml_jni_shim_test")


def _find_jni() -> list:
    home = os.environ.get("JAVA_HOME")
    cands = [home] if home else []
    cands += glob.glob("/usr/lib/jvm/*")
    for c in cands:
        inc = os.path.join(c, "include")
        if os.path.exists(os.path.join(inc, "jni.h")):
            return [inc, os.path.join(inc, "linux")]
    return []


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--test", action="store_true")
    a = ap.parse_args()
    exe = build(verbose=True)
    if a.test:
        return subprocess.call([exe])
    return 0


if __name__ == "__main__":
    sys.exit(main())
