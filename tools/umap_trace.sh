#!/bin/bash
# Kernel trace of one UMAP fit at the north-star shape (ROWS, default 20M x 128).
set -o pipefail
mkdir -p gpurun_out/umap_trace/raw
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/umap_trace/raw -o run -- python3 tools/umap_phases.py --rows ${ROWS:-20000000} > gpurun_out/umap_trace/log.txt 2>&1 || { tail -20 gpurun_out/umap_trace/log.txt; exit 1; }
python3 tools/trace_summary.py gpurun_out/umap_trace | head -32
