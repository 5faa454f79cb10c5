#!/bin/bash
# Test tiers (the role of the reference's python/run_test.sh + CI jobs):
#   ci/run_tests.sh lint    — stdlib lint gate (ci/lint.py)
#   ci/run_tests.sh cpu     — every non-GPU test (CPU reference paths, gloo multi-rank, fake pyspark)
#   ci/run_tests.sh gpu     — the MI355X tier (run on a GPU box: kernels vs CPU oracles, smoke)
#   ci/run_tests.sh sanitize — host ASan/UBSan build of the JNI shim + C-ABI checks (no GPU)
#   ci/run_tests.sh all     — lint + sanitize + cpu
set -euo pipefail
cd "$(dirname "$0")/.."
tier=${1:-all}
case "$tier" in
  lint) python ci/lint.py ;;
  cpu) python -m pytest tests/ -x -q -m "not gpu" -n "${PYTEST_WORKERS:-4}" ;;
  gpu) python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread ;;
  sanitize) bash native/tests/run_sanitizers.sh ;;
  all) python ci/lint.py && bash native/tests/run_sanitizers.sh &&
       python -m pytest tests/ -x -q -m "not gpu" -n "${PYTEST_WORKERS:-4}" ;;
  *) echo "usage: $0 [lint|cpu|gpu|sanitize|all]"; exit 2 ;;
esac
