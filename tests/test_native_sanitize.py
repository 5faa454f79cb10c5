"""Host-side sanitizer tier (SURVEY §5 race detection / sanitizers): the JNI shim's argument
marshalling and the C-ABI validation built with -fsanitize=address,undefined against a host stub
of the srml_capi_* entry points and executed (native/tests/run_sanitizers.sh). GPU sanitizers are
not available on the MI355X pool, so the device side is covered by the GPU tier's oracles."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which(os.environ.get("CXX", "g++")) is None, reason="no host C++ compiler")
def test_asan_ubsan_jni_shim_and_capi_checks(tmp_path):
    env = dict(os.environ, SRML_SANITIZE_OUT=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "native", "tests", "run_sanitizers.sh")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "jni shim: ok" in r.stdout and "capi checks: ok" in r.stdout
