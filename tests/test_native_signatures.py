"""Every entry point the Python layer launches through ``native.call`` has a declared ctypes
signature (ops/native.py SIGNATURES): without one ctypes would pass 64-bit pointers and sizes as
C ints; ``native.call`` refuses such names, and this test finds them before a GPU run does."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_called_entry_points_have_signatures():
    from spark_rapids_ml_nai_amd.ops.native import SIGNATURES

    names, prefixes = set(), set()
    for f in glob.glob(os.path.join(ROOT, "spark_rapids_ml_nai_amd", "**", "*.py"), recursive=True):
        src = open(f).read()
        for m in re.finditer(r'native\.call\(\s*"(srml_[A-Za-z0-9_]+)"(\s*\+)?', src):
            (prefixes if m.group(2) else names).add(m.group(1))
    assert names, "no native.call sites found"
    assert sorted(n for n in names if n not in SIGNATURES) == []
    for p in prefixes:  # dtype-suffixed families: both variants declared
        assert {p + "f32", p + "f64"} <= set(SIGNATURES), p
    # the names chosen at run time
    for n in ("srml_xtv_mfma_f32", "srml_xtv2_f32", "srml_col_moments_f32", "srml_col_moments_f64"):
        assert n in SIGNATURES
