#!/bin/bash
# fp16 centred IVF candidate kernel: numerics tests, the 20M probe, then the UMAP trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -k "knn_lists or knn_graph_ivf" -x -v --timeout 240 \
    --timeout-method thread > gpurun_out/knnf16_pytest.log 2>&1 || { tail -40 gpurun_out/knnf16_pytest.log; exit 1; }
tail -3 gpurun_out/knnf16_pytest.log
timeout -k 10 300 python3 tools/ivf_probe.py > gpurun_out/ivf_probe_f16.log 2>&1 || { tail -20 gpurun_out/ivf_probe_f16.log; exit 1; }
tail -1 gpurun_out/ivf_probe_f16.log
