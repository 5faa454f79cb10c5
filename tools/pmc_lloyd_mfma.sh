#!/bin/bash
# PMC passes over the MFMA small-k Lloyd step (tools/lloyd_mfma_bench.py at 10M x 64, k = 20):
# VALU / MFMA / LDS / VMEM activity, then L2 traffic and LDS conflicts — one rocprofv3 run each.
set -o pipefail
mkdir -p gpurun_out/pmclm
export TMPDIR=/tmp
export ROWS=10000000
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS -d gpurun_out/pmclm/p1 -o p1 --output-format csv -- python3 tools/lloyd_mfma_bench.py > gpurun_out/pmclm/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/pmclm/p2 -o p2 --output-format csv -- python3 tools/lloyd_mfma_bench.py > gpurun_out/pmclm/p2.log 2>&1 || exit 1
python3 tools/pmc_summary.py "lloyd_mfma_kernel" gpurun_out/pmclm > gpurun_out/pmclm/summary.json
rm -rf gpurun_out/pmclm/p1 gpurun_out/pmclm/p2
cat gpurun_out/pmclm/summary.json
