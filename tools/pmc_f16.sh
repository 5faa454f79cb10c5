#!/bin/bash
# PMC passes over the fp16 certified KMeans filter microbench (m=250000, n=3000, k=1000 random-row
# centres): MFMA / wave-state, L2 / LDS, and memory-pipe counter groups (one rocprofv3 run each).
set -o pipefail
mkdir -p gpurun_out/pmc16
export TMPDIR=/tmp
K="--only nearest_f16 --m 250000"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_WAIT_INST_LDS -d gpurun_out/pmc16/p1 -o p1 --output-format csv -- python3 tools/kbench.py $K > gpurun_out/pmc16/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/pmc16/p2 -o p2 --output-format csv -- python3 tools/kbench.py $K > gpurun_out/pmc16/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d gpurun_out/pmc16/p3 -o p3 --output-format csv -- python3 tools/kbench.py $K > gpurun_out/pmc16/p3.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc16/p4 -o p4 --output-format csv -- python3 tools/kbench.py $K > gpurun_out/pmc16/p4.log 2>&1 || { tail -5 gpurun_out/pmc16/p4.log; }
python3 tools/pmc_summary.py "glds_kernel<true, 1," gpurun_out/pmc16 > gpurun_out/pmc16/summary.json
cat gpurun_out/pmc16/summary.json
timeout -k 10 120 python3 tools/kbench.py --only nearest_f16,sums > gpurun_out/kbench_f16.json 2>&1 || exit 1
tail -1 gpurun_out/kbench_f16.json
