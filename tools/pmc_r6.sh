#!/bin/bash
# Counter evidence (round 6): the fused RF node split (rf_node_split_kernel) in the RFC bench fit,
# and the LogReg evaluations (full loss/gradient passes vs line-search margins-only passes) in the
# LogReg bench fit. Per workload: a kernel-trace --stats run (per-kernel time), then PMC passes
# (wave states / LDS; HBM fetch bytes + L2 hit). Summaries under gpurun_out/pmc6/.
set -o pipefail
mkdir -p gpurun_out/pmc6
export TMPDIR=/tmp
for W in random_forest_classifier logistic_regression; do
  B="python3 bench.py --steps 1 --warmup 0 --algos $W --no-transform --no-quality"
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc6/$W/t -o t --output-format csv -- $B > gpurun_out/pmc6/$W.t.log 2>&1 || { tail -5 gpurun_out/pmc6/$W.t.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/pmc6/$W/p1 -o p1 --output-format csv -- $B > gpurun_out/pmc6/$W.p1.log 2>&1 || { tail -5 gpurun_out/pmc6/$W.p1.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d gpurun_out/pmc6/$W/p2 -o p2 --output-format csv -- $B > gpurun_out/pmc6/$W.p2.log 2>&1 || { tail -5 gpurun_out/pmc6/$W.p2.log; exit 1; }
done
python3 tools/pmc_r6_summary.py gpurun_out/pmc6 > gpurun_out/pmc6/summary.json && cat gpurun_out/pmc6/summary.json
