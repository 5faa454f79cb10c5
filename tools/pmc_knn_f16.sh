#!/bin/bash
# PMC passes over the fp16 centred IVF kNN tile kernel (tools/knn_lists_bench.py, 4M x 128).
set -o pipefail
mkdir -p gpurun_out/pmckg
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/knn_lists_bench.py > gpurun_out/pmckg/plain.log 2>&1 || exit 1
cat gpurun_out/pmckg/plain.log | grep knn_lists
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS -d gpurun_out/pmckg/p1 -o p1 --output-format csv -- python3 tools/knn_lists_bench.py > gpurun_out/pmckg/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU -d gpurun_out/pmckg/p2 -o p2 --output-format csv -- python3 tools/knn_lists_bench.py > gpurun_out/pmckg/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmckg/p3 -o p3 --output-format csv -- python3 tools/knn_lists_bench.py > gpurun_out/pmckg/p3.log 2>&1 || exit 1
python3 tools/pmc_summary.py "knn_lists_f16_kernel" gpurun_out/pmckg > gpurun_out/pmckg/summary.json
cat gpurun_out/pmckg/summary.json
