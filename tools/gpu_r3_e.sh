#!/bin/bash
# Round-3 batch E: packed regression cells in the wide RF histogram (GPU tests + regressor trace,
# packed vs exact fixed point).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_fp64_topk.py tests/test_ops_gpu.py tests/test_models_api.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rf_ or forest" > gpurun_out/pytest_e.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_e.log; exit 1; }
tail -2 gpurun_out/pytest_e.log
ALGOS=random_forest_regressor TAG=rfr_packed bash tools/gpu_trace_algo.sh \
 && SRML_RF_PACK=0 ALGOS=random_forest_regressor TAG=rfr_unpacked bash tools/gpu_trace_algo.sh || exit 1
