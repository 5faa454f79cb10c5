"""docs/api.md is generated from the package (tools/gen_api_docs.py) and must be current: a public
class or Param added without regenerating the reference fails here."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_api_reference_is_current():
    env = dict(os.environ, SRML_FORCE_CPU="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_api_docs.py"), "--check"], env=env,
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
