#!/bin/bash
# Round-3 targeted checks: new kernels' GPU tests, then the RF item-order A/B traces.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_qn.py tests/test_sparse.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ivf_search or knn_lists or cd_gram or loss_grad" > gpurun_out/pytest_r3.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_r3.log; exit 1; }
tail -2 gpurun_out/pytest_r3.log
ALGOS=random_forest_regressor TAG=rfr_chunkmajor bash tools/gpu_trace_algo.sh && ALGOS=random_forest_classifier TAG=rfc_chunkmajor bash tools/gpu_trace_algo.sh && SRML_RF_ITEM_ORDER=node ALGOS=random_forest_regressor TAG=rfr_nodemajor bash tools/gpu_trace_algo.sh
