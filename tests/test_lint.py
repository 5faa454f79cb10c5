"""The repository lint gate (ci/lint.py) is part of the CPU test tier."""
import os
import subprocess
import sys


def test_lint_gate_clean():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "ci", "lint.py")], capture_output=True, text=True,
                       cwd=root, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:]
