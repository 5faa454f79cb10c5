#!/bin/bash
# Round-5 UMAP 20M x 128: host-profiled fit with per-phase times, then a kernel trace of a fit
# with the device-idle gaps listed.
set -o pipefail
mkdir -p gpurun_out/umap_trace/raw
export TMPDIR=/tmp

timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/umap_trace/raw -o run -- python3 tools/umap_phases.py --rows 20000000 --no-profile > gpurun_out/umap_trace/log.txt 2>&1 || { tail -20 gpurun_out/umap_trace/log.txt; exit 1; }
TRACE_AFTER_GAP_MS=1000 TRACE_GAPS=25 python3 tools/trace_summary.py gpurun_out/umap_trace > gpurun_out/umap_trace_summary.txt
rm -rf gpurun_out/umap_trace/raw
grep -v amdgpu gpurun_out/umap_trace/log.txt | head -5
