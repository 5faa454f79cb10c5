#!/bin/bash
# Fused RF split with 8 rows in flight per wave: tests + RFC per-level timing (two runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_rf_levels.py \
  > gpurun_out/t_nsu.log 2>&1 || { tail -30 gpurun_out/t_nsu.log; exit 1; }
tail -n 1 gpurun_out/t_nsu.log
for rep in 1 2; do
  timeout -k 10 200 python -u tools/rf_levels.py 1000000 > gpurun_out/rfl_nsu_$rep.txt 2>&1 || exit 1
  grep fit_s gpurun_out/rfl_nsu_$rep.txt
done
