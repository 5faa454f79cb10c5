#!/bin/bash
# RF wide record-layout histogram + KMeans 256x128 3-product tile: GPU equivalence tests, the
# certified-pass A/B (kbench) and per-level traces of the regressor with the wide kernel from
# density 3% / 20% / 60%.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_fp64_topk.py tests/test_ops_gpu.py tests/test_qn.py tests/test_umap_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rf_ or nearest or kmeans or split or graph or qn_kernel or label_sort or ivf or cluster_sums or radix or fuzzy or umap" > gpurun_out/pytest_rf.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_rf.log; exit 1; }
tail -2 gpurun_out/pytest_rf.log
timeout -k 10 300 python3 tools/kbench.py --only nearest_certified > gpurun_out/kb_bn128.json 2>&1 && cat gpurun_out/kb_bn128.json \
 && SRML_SPLIT_BN3=256 timeout -k 10 300 python3 tools/kbench.py --only nearest_certified > gpurun_out/kb_bn256.json 2>&1 && cat gpurun_out/kb_bn256.json \
 && ALGOS=random_forest_regressor TAG=rfr_wide03 bash tools/gpu_trace_algo.sh \
 && SRML_RF_IL_DENSITY=0.2 ALGOS=random_forest_regressor TAG=rfr_wide20 bash tools/gpu_trace_algo.sh \
 && SRML_RF_IL_DENSITY=0.6 ALGOS=random_forest_regressor TAG=rfr_wide60 bash tools/gpu_trace_algo.sh \
 && SRML_RF_IL_DENSITY=0.2 ALGOS=random_forest_classifier TAG=rfc_wide20 bash tools/gpu_trace_algo.sh \
 && ALGOS=random_forest_classifier TAG=rfc_wide03 bash tools/gpu_trace_algo.sh || exit 1
# LogReg 125k-row (8-GPU per-rank) proxy: QN batches replayed from a HIP graph vs eager
SRML_QN_GRAPH=0 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --rows 125000 --algos logistic_regression --no-transform > gpurun_out/lr125k_eager.json 2> gpurun_out/lr125k_eager.err && tail -1 gpurun_out/lr125k_eager.json \
 && timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --rows 125000 --algos logistic_regression --no-transform > gpurun_out/lr125k_graph.json 2> gpurun_out/lr125k_graph.err && tail -1 gpurun_out/lr125k_graph.json
