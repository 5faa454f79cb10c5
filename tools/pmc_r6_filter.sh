#!/bin/bash
# Round-6 PMC of the fp16 certified KMeans filter (kbench nearest_f16 at m = 250000, n = 3000,
# k = 1000) and of the small-k MFMA Lloyd step (10M x 64, k = 20): one rocprofv3 run per pass.
set -o pipefail
mkdir -p gpurun_out/pmc6f gpurun_out/pmc6l
export TMPDIR=/tmp
K="--only nearest_f16 --m 250000"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_WAIT_INST_LDS -d gpurun_out/pmc6f/p1 -o p1 --output-format csv -- python3 tools/kbench.py $K > gpurun_out/pmc6f/p1.log 2>&1 || { tail -5 gpurun_out/pmc6f/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/pmc6f/p2 -o p2 --output-format csv -- python3 tools/kbench.py $K > gpurun_out/pmc6f/p2.log 2>&1 || { tail -5 gpurun_out/pmc6f/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d gpurun_out/pmc6f/p3 -o p3 --output-format csv -- python3 tools/kbench.py $K > gpurun_out/pmc6f/p3.log 2>&1 || { tail -5 gpurun_out/pmc6f/p3.log; exit 1; }
python3 tools/pmc_summary.py "nearest_centroid_split_glds_kernel<true" gpurun_out/pmc6f > gpurun_out/pmc6f/summary.json
cat gpurun_out/pmc6f/summary.json | head -60
timeout -k 10 120 python3 tools/kbench.py --only nearest_f16 > gpurun_out/pmc6f/kbench_f16.json 2>&1 || exit 1
tail -1 gpurun_out/pmc6f/kbench_f16.json
export ROWS=10000000
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS -d gpurun_out/pmc6l/p1 -o p1 --output-format csv -- python3 tools/lloyd_mfma_bench.py > gpurun_out/pmc6l/p1.log 2>&1 || { tail -5 gpurun_out/pmc6l/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/pmc6l/p2 -o p2 --output-format csv -- python3 tools/lloyd_mfma_bench.py > gpurun_out/pmc6l/p2.log 2>&1 || { tail -5 gpurun_out/pmc6l/p2.log; exit 1; }
python3 tools/pmc_summary.py "lloyd_mfma_kernel" gpurun_out/pmc6l > gpurun_out/pmc6l/summary.json
cat gpurun_out/pmc6l/summary.json | head -40
rm -rf gpurun_out/pmc6f/p1 gpurun_out/pmc6f/p2 gpurun_out/pmc6f/p3 gpurun_out/pmc6l/p1 gpurun_out/pmc6l/p2
