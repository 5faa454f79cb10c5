#!/bin/bash
# Row-major bins for sparse RF levels: equivalence tests, then the RFC bench fit at thresholds 0 / 2000 / always.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_rf_levels.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/rm_t.log 2>&1 || { tail -20 gpurun_out/rm_t.log; exit 1; }
tail -1 gpurun_out/rm_t.log
for t in 0 2000 1000000000; do
  SRML_RF_ROWMAJOR_ROWS=$t timeout -k 10 200 python -u tools/rf_levels.py 1000000 > gpurun_out/rm_$t.txt 2>&1 || exit 1
  echo "rm=$t $(grep workload gpurun_out/rm_$t.txt)"
done
