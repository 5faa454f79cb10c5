#!/bin/bash
# cProfile host view of several headline fits at a given per-rank row count (default 125000 = 1M/8).
set -o pipefail
mkdir -p gpurun_out
ROWS=${ROWS:-125000}
for a in ${ALGOS:-pca kmeans logistic_regression random_forest_classifier}; do
  timeout -k 10 200 python -u tools/fit_profile.py $a --rows $ROWS --top 30 > gpurun_out/fitprof_$a.txt 2>&1 || { tail -20 gpurun_out/fitprof_$a.txt; exit 1; }
  grep "fit wall" gpurun_out/fitprof_$a.txt | sed "s/^/$a /"
done
