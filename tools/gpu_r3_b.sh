#!/bin/bash
# Round-3 batch B: GPU tests of the new kernels (wide RF histogram on 32/64-B records, label sort,
# radix sort, kNN refine-sort), then traces: RF regressor record size / density, KMeans Lloyd with
# the 256x128 vs 256x256 3-product tile, LogReg at the 125k-row per-rank size.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_fp64_topk.py tests/test_ops_gpu.py tests/test_qn.py tests/test_umap_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rf_ or nearest or kmeans or split or graph or label_sort or radix or refine or fuzzy or umap or knn" > gpurun_out/pytest_b.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_b.log; exit 1; }
tail -2 gpurun_out/pytest_b.log
ALGOS=random_forest_regressor TAG=rfr_w64_d12 bash tools/gpu_trace_algo.sh \
 && SRML_RF_REC_BYTES=32 ALGOS=random_forest_regressor TAG=rfr_w32_d12 bash tools/gpu_trace_algo.sh \
 && SRML_RF_IL_DENSITY=0.3 ALGOS=random_forest_regressor TAG=rfr_w64_d30 bash tools/gpu_trace_algo.sh \
 && ALGOS=kmeans TAG=km_bn128 bash tools/gpu_trace_algo.sh \
 && SRML_SPLIT_BN3=256 ALGOS=kmeans TAG=km_bn256 bash tools/gpu_trace_algo.sh \
 && BENCH_EXTRA="--rows 125000" ALGOS=logistic_regression TAG=lr125k bash tools/gpu_trace_algo.sh || exit 1
