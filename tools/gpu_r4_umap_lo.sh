#!/bin/bash
# UMAP list-order + pull epochs: GPU tests, then the 20M kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_umap_gpu.py tests/test_ops_gpu.py -k "umap" -x -q --timeout 240 \
    --timeout-method thread > gpurun_out/umap_lo_pytest.log 2>&1 || { tail -30 gpurun_out/umap_lo_pytest.log; exit 1; }
tail -2 gpurun_out/umap_lo_pytest.log
bash tools/umap_trace.sh
