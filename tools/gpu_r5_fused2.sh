#!/bin/bash
# Fused RF split + LDS transpose: tests, per-level timing, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_rf_levels.py \
  > gpurun_out/t_fused2.log 2>&1 || { tail -30 gpurun_out/t_fused2.log; exit 1; }
timeout -k 10 300 python -u tools/rf_levels.py 1000000 > gpurun_out/rfl_fused2.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o rfc -- python3 tools/rf_levels.py 1000000 \
  > gpurun_out/prof_fused.log 2>&1 || exit 1
tail -n 2 gpurun_out/t_fused2.log
grep fit_s gpurun_out/rfl_fused2.txt
