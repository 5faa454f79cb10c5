#!/bin/bash
# Kernel trace of the 125k-row per-rank proxy for PCA and LinReg: what runs after the Gram.
set -o pipefail
mkdir -p gpurun_out/r6z
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6z/tr -o tr -- python3 bench.py --rows 125000 --steps 1 --warmup 1 --algos pca,linear_regression --no-transform > gpurun_out/r6z/b.json 2> gpurun_out/r6z/b.err || { tail -20 gpurun_out/r6z/b.err; exit 1; }
gzip -f gpurun_out/r6z/tr/*kernel_trace.csv
