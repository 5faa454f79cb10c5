"""No kernel of the HIP library spills to scratch on gfx950: every source is compiled with the
compiler's per-kernel resource remarks and each kernel's ScratchSize must be 0 (a spill is a per-lane
round trip through memory inside the hot loops; dynamic indexing of a register array or a loop the
compiler cannot unroll is the usual cause)."""
import glob
import os
import re
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "spark_rapids_ml_nai_amd", "ops",
                    "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _scratch_kernels(src: str, tmp: str):
    out = os.path.join(tmp, os.path.basename(src) + ".o")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", out,
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    bad, name = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and int(m.group(1)) > 0:
            bad.append((os.path.basename(src), name, int(m.group(1))))
    return bad


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_no_kernel_spills_to_scratch(tmp_path):
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    assert srcs
    with ThreadPoolExecutor(max_workers=min(6, os.cpu_count() or 1)) as ex:
        found = [b for bad in ex.map(lambda s: _scratch_kernels(s, str(tmp_path)), srcs) for b in bad]
    assert found == [], found
