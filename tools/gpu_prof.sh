#!/bin/bash
# rocprofv3 kernel-trace stats of the headline bench (1 GPU); summary CSVs land in gpurun_out/prof.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ALGOS=${ALGOS:-all}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 1 --warmup 1 --algos $ALGOS > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || { echo "prof failed"; tail -30 gpurun_out/prof_bench.err; exit 1; }
cat gpurun_out/prof_bench.json
find gpurun_out/prof -name "*kernel_stats.csv" | head
