#!/bin/bash
# UMAP inverted-list-order pipeline: GPU tests, then the 20M kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_umap_gpu.py -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/umap_lo_pytest.log 2>&1 || { tail -30 gpurun_out/umap_lo_pytest.log; exit 1; }
tail -2 gpurun_out/umap_lo_pytest.log
bash tools/umap_trace.sh
