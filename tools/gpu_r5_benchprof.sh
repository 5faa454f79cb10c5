#!/bin/bash
# Kernel statistics of one warm bench step (all eight workloads) after the fused RF split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof_bench
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- \
  python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_bench/log.txt 2>&1 || { tail -20 gpurun_out/prof_bench/log.txt; exit 1; }
find gpurun_out/prof_bench -name "*kernel_stats.csv" | head -3
