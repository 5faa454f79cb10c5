#!/bin/bash
# Round 6: per-workload glue count. One rocprofv3 kernel-trace run per bench workload
# (--steps 1 --warmup 1, transforms and quality included, as the full-bench trace), listing the
# torch (at::native / rocprim) launches of each so the remaining glue can be attributed.
set -o pipefail
mkdir -p gpurun_out/r6j
export TMPDIR=/tmp
for A in kmeans pca linear_regression linear_regression_elasticnet linear_regression_ridge logistic_regression random_forest_classifier random_forest_regressor; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r6j/p_$A -o prof --output-format csv -- python3 bench.py --steps 1 --warmup 1 --algos $A > gpurun_out/r6j/$A.json 2> gpurun_out/r6j/$A.err || { tail -20 gpurun_out/r6j/$A.err; exit 1; }
  python3 tools/glue_summary.py gpurun_out/r6j/p_$A $A >> gpurun_out/r6j/glue.txt || exit 1
  rm -rf gpurun_out/r6j/p_$A/*/*kernel_trace.csv
done
cat gpurun_out/r6j/glue.txt
