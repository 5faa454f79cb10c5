#!/bin/bash
# RF record-layout histogram: GPU equivalence tests, then per-level traces at IL depth 2 / 0 / off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_fp64_topk.py tests/test_ops_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rf_" > gpurun_out/pytest_rf.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_rf.log; exit 1; }
tail -2 gpurun_out/pytest_rf.log
ALGOS=random_forest_regressor TAG=rfr_il2 bash tools/gpu_trace_algo.sh && SRML_RF_IL_DEPTH=0 ALGOS=random_forest_regressor TAG=rfr_il0 bash tools/gpu_trace_algo.sh && ALGOS=random_forest_classifier TAG=rfc_il2 bash tools/gpu_trace_algo.sh
