#!/bin/bash
# Round-3 batch C: wide RF histogram on paired 64-B records (GPU equivalence tests + regressor
# trace), certified KMeans pass with s_setprio around the MFMA clusters (256x256 and 256x128).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_fp64_topk.py tests/test_ops_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rf_ or certified" > gpurun_out/pytest_c.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_c.log; exit 1; }
tail -2 gpurun_out/pytest_c.log
ALGOS=random_forest_regressor TAG=rfr_pair64 bash tools/gpu_trace_algo.sh \
 && SRML_SPLIT_PRIO=1 SRML_SPLIT_BN3=256 ALGOS=kmeans TAG=km_prio256 bash tools/gpu_trace_algo.sh \
 && SRML_SPLIT_PRIO=1 ALGOS=kmeans TAG=km_prio128 bash tools/gpu_trace_algo.sh || exit 1
