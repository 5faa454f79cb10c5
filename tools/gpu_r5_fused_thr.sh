#!/bin/bash
# RFC bench fit vs the fused / row-major level thresholds (alternating, two runs each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/fused_thr.txt
for rep in 1 2; do
  for thr in 10000 5000 20000; do
    SRML_RF_FUSED_ROWS=$thr SRML_RF_ROWMAJOR_ROWS=$thr timeout -k 10 200 python -u tools/rf_levels.py 1000000 \
      > gpurun_out/rfl_thr_$thr.txt 2>&1 || exit 1
    echo "thr=$thr $(grep fit_s gpurun_out/rfl_thr_$thr.txt)" >> gpurun_out/fused_thr.txt
  done
done
cat gpurun_out/fused_thr.txt
