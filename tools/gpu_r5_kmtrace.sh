#!/bin/bash
# Kernel trace of the KMeans k=1000 bench fit (1M x 3000): per-kernel totals of the timed step.
set -o pipefail
mkdir -p gpurun_out/kmtrace/raw
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kmtrace/raw -o run -- python3 bench.py --steps 1 --warmup 1 --algos kmeans --no-transform --no-quality > gpurun_out/kmtrace/bench.json 2> gpurun_out/kmtrace/bench.err || { tail -20 gpurun_out/kmtrace/bench.err; exit 1; }
TRACE_GAPS=8 python3 tools/trace_summary.py gpurun_out/kmtrace > gpurun_out/kmtrace_summary.txt
rm -rf gpurun_out/kmtrace/raw
