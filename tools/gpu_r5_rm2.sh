#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for t in 0 1000 4000 10000 30000; do
  SRML_RF_ROWMAJOR_ROWS=$t timeout -k 10 200 python -u tools/rf_levels.py 1000000 > gpurun_out/rm_$t.txt 2>&1 || exit 1
  echo "rm=$t $(grep workload gpurun_out/rm_$t.txt)"
done
SRML_RF_ROWMAJOR_ROWS=4000 timeout -k 10 200 python -u tools/rf_levels.py 1000000 random_forest_regressor > gpurun_out/rm_rfr.txt 2>&1 || exit 1
echo "rfr rm=4000 $(grep workload gpurun_out/rm_rfr.txt)"
