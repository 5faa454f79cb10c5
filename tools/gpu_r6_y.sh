#!/bin/bash
# Kernel trace of the 125k-row per-rank proxy (KMeans, LogReg, RFC): device busy vs idle per fit.
set -o pipefail
mkdir -p gpurun_out/r6y
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6y/tr -o tr -- python3 bench.py --rows 125000 --steps 1 --warmup 1 --algos kmeans,logistic_regression,random_forest_classifier --no-transform > gpurun_out/r6y/b.json 2> gpurun_out/r6y/b.err || { tail -20 gpurun_out/r6y/b.err; exit 1; }
python3 tools/trace_gaps.py gpurun_out/r6y/tr > gpurun_out/r6y/gaps.txt && cat gpurun_out/r6y/gaps.txt
gzip -f gpurun_out/r6y/tr/*kernel_trace.csv
