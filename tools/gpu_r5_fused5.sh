#!/bin/bash
# Fused RF split (uniform / multi-row variants, precedence over the record layout): tests, RFC + north-star timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_rf_levels.py \
  > gpurun_out/t_fused5.log 2>&1 || { tail -30 gpurun_out/t_fused5.log; exit 1; }
timeout -k 10 300 python -u tools/rf_levels.py 1000000 > gpurun_out/rfl_fused5.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/rf_levels.py 50000000 northstar_rf > gpurun_out/ns_rf_f4_default.txt 2>&1 || exit 1
SRML_RF_FUSED_ROWS=1e12 timeout -k 10 400 python -u tools/rf_levels.py 50000000 northstar_rf \
  > gpurun_out/ns_rf_f4_allfused.txt 2>&1 || exit 1
tail -n 2 gpurun_out/t_fused5.log
grep -h fit_s gpurun_out/rfl_fused5.txt gpurun_out/ns_rf_f4_default.txt gpurun_out/ns_rf_f4_allfused.txt
