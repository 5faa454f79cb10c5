#!/bin/bash
# Fused small-node RF split: numerics tests, per-level timing fused vs unfused, RF test subset.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_rf_levels.py \
  > gpurun_out/t_fused.log 2>&1 || { tail -30 gpurun_out/t_fused.log; exit 1; }
timeout -k 10 300 python -u tools/rf_levels.py 1000000 > gpurun_out/rfl_fused.txt 2>&1 || exit 1
SRML_RF_FUSED_ROWS=0 timeout -k 10 300 python -u tools/rf_levels.py 1000000 > gpurun_out/rfl_unfused.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  -k "forest or rf_ or Forest or tree" tests/ > gpurun_out/t_rf_all.log 2>&1 || { tail -30 gpurun_out/t_rf_all.log; exit 1; }
tail -3 gpurun_out/t_fused.log gpurun_out/t_rf_all.log
head -2 gpurun_out/rfl_fused.txt gpurun_out/rfl_unfused.txt | grep fit_s
