#!/bin/bash
# PMC passes over the certified 3-product KMeans pass (kbench nearest_certified, m=250000,
# n=3000, k=1000): MFMA busy, wait breakdown, L2 hit, LDS conflicts. One rocprofv3 run per
# counter group. KERNEL selects the dispatches summarised.
set -o pipefail
mkdir -p gpurun_out/pmc_cert
export TMPDIR=/tmp
K="${KERNEL:-glds_kernel<true, 3, true}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS -d gpurun_out/pmc_cert/p1 -o p1 --output-format csv -- python3 tools/kbench.py --only nearest_certified --m 250000 > gpurun_out/pmc_cert/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/pmc_cert/p2 -o p2 --output-format csv -- python3 tools/kbench.py --only nearest_certified --m 250000 > gpurun_out/pmc_cert/p2.log 2>&1 || exit 1
python3 tools/pmc_summary.py "$K" gpurun_out/pmc_cert > gpurun_out/pmc_cert/summary.json
cat gpurun_out/pmc_cert/summary.json
