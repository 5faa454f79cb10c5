#!/bin/bash
# PMC passes over the fused small-k Lloyd step (tools/lloyd_small_bench.py: 10M x 64, k = 20 with
# sums, then the search alone) — VALU / MFMA / LDS activity, L2 traffic — one rocprofv3 run per group.
set -o pipefail
mkdir -p gpurun_out/pmcls
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU -d gpurun_out/pmcls/p1 -o p1 --output-format csv -- python3 tools/lloyd_small_bench.py > gpurun_out/pmcls/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/pmcls/p2 -o p2 --output-format csv -- python3 tools/lloyd_small_bench.py > gpurun_out/pmcls/p2.log 2>&1 || exit 1
python3 tools/pmc_summary.py "lloyd_small_kernel<16, 24>" gpurun_out/pmcls > gpurun_out/pmcls/summary.json
cat gpurun_out/pmcls/summary.json
tail -3 gpurun_out/pmcls/p2.log
