#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -k "knn_lists or knn_graph_ivf" -x -q --timeout 240 \
    --timeout-method thread > gpurun_out/knnf16_pytest.log 2>&1 || { tail -40 gpurun_out/knnf16_pytest.log; exit 1; }
tail -2 gpurun_out/knnf16_pytest.log
timeout -k 10 120 python3 tools/knn_lists_bench.py > gpurun_out/knnb.log 2>&1 || { tail -20 gpurun_out/knnb.log; exit 1; }
grep knn_lists gpurun_out/knnb.log
timeout -k 10 300 python3 tools/ivf_probe.py > gpurun_out/ivf_probe_f16.log 2>&1 || { tail -20 gpurun_out/ivf_probe_f16.log; exit 1; }
tail -1 gpurun_out/ivf_probe_f16.log
