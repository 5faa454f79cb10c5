#!/bin/bash
# GPU session: new-kernel tests -> UMAP tests on the device -> north-star configs (1 GPU).
# Every step has its own time limit; the first failure ends the session.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SCALE_LR=${SCALE_LR:-0.25}
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "knn_lists or knn or ivf" -x -v --timeout 120 --timeout-method thread > gpurun_out/ns_pytest_kernels.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/ns_pytest_kernels.log; exit 1; }
tail -2 gpurun_out/ns_pytest_kernels.log
timeout -k 10 400 python -u -m pytest tests/test_umap.py -x -v --timeout 200 --timeout-method thread -k "not two_ranks" > gpurun_out/ns_pytest_umap.log 2>&1 || { echo "umap tests failed"; tail -30 gpurun_out/ns_pytest_umap.log; exit 1; }
tail -2 gpurun_out/ns_pytest_umap.log
rm -f gpurun_out/northstar_1gpu.jsonl
timeout -k 10 300 python -u tools/northstar.py --configs pca,kmeans --out gpurun_out/northstar_1gpu.jsonl > gpurun_out/ns_a.log 2>&1 || { echo "northstar a failed"; tail -30 gpurun_out/ns_a.log; exit 1; }
timeout -k 10 300 python -u tools/northstar.py --configs umap --scale 0.1 --out gpurun_out/northstar_1gpu.jsonl > gpurun_out/ns_b.log 2>&1 || { echo "northstar umap failed"; tail -30 gpurun_out/ns_b.log; exit 1; }
timeout -k 10 400 python -u tools/northstar.py --configs logreg --scale $SCALE_LR --out gpurun_out/northstar_1gpu.jsonl > gpurun_out/ns_c.log 2>&1 || { echo "northstar logreg failed"; tail -30 gpurun_out/ns_c.log; exit 1; }
timeout -k 10 400 python -u tools/northstar.py --configs rf --scale 0.1 --out gpurun_out/northstar_1gpu.jsonl > gpurun_out/ns_d.log 2>&1 || { echo "northstar rf failed"; tail -30 gpurun_out/ns_d.log; exit 1; }
cat gpurun_out/northstar_1gpu.jsonl
