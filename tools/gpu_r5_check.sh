#!/bin/bash
# Round-5 validation on one MI355X: every GPU test, the smoke step, the round-5 native-path trace
# and the RFC kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r5.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r5.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5.log 2>&1 || { tail -20 gpurun_out/smoke_r5.log; exit 1; }
tail -1 gpurun_out/smoke_r5.log
bash tools/gpu_r5_native.sh > gpurun_out/np5_out.txt 2>&1; echo "native check rc $?"
head -3 gpurun_out/np5/check.txt
bash tools/gpu_r5_rftrace.sh || exit 1
head -30 gpurun_out/rftrace_summary.txt
