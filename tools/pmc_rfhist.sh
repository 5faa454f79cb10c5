#!/bin/bash
# PMC passes over the RF histogram microbench (root level, 1M rows x 1000 of 3000 features).
set -o pipefail
mkdir -p gpurun_out/pmc_rf
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/kbench.py --only rfhist > gpurun_out/pmc_rf/time.json 2>&1 || exit 1
cat gpurun_out/pmc_rf/time.json | tail -1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d gpurun_out/pmc_rf/p1 -o p1 --output-format csv -- python3 tools/kbench.py --only rfhist > gpurun_out/pmc_rf/p1.log 2>&1 || { tail -5 gpurun_out/pmc_rf/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU -d gpurun_out/pmc_rf/p2 -o p2 --output-format csv -- python3 tools/kbench.py --only rfhist > gpurun_out/pmc_rf/p2.log 2>&1 || { tail -5 gpurun_out/pmc_rf/p2.log; exit 1; }
python3 tools/pmc_summary.py "rf_hist_kernel<true, false>" gpurun_out/pmc_rf > gpurun_out/pmc_rf/summary_reg.json
python3 tools/pmc_summary.py "rf_hist_kernel<false, false>" gpurun_out/pmc_rf > gpurun_out/pmc_rf/summary_clf.json
cat gpurun_out/pmc_rf/summary_reg.json gpurun_out/pmc_rf/summary_clf.json
