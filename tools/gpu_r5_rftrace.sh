#!/bin/bash
# Kernel trace of the RFC bench-shape fit (warm-up + timed fit in tools/rf_levels.py).
set -o pipefail
mkdir -p gpurun_out/rftrace/raw
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rftrace/raw -o run -- python3 tools/rf_levels.py 1000000 > gpurun_out/rftrace/log.txt 2>&1 || { tail -20 gpurun_out/rftrace/log.txt; exit 1; }
TRACE_GAPS=10 python3 tools/trace_summary.py gpurun_out/rftrace > gpurun_out/rftrace_summary.txt
rm -rf gpurun_out/rftrace/raw
