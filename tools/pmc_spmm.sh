#!/bin/bash
# PMC passes over the CSR SpMM (tools/spmm_bench.py, 4M rows).
set -o pipefail
mkdir -p gpurun_out/pmcsp
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/spmm_bench.py > gpurun_out/pmcsp/plain.log 2>&1 || { tail gpurun_out/pmcsp/plain.log; exit 1; }
grep -E "rows|spmm" gpurun_out/pmcsp/plain.log
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_SALU -d gpurun_out/pmcsp/p1 -o p1 --output-format csv -- python3 tools/spmm_bench.py > gpurun_out/pmcsp/p1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum -d gpurun_out/pmcsp/p2 -o p2 --output-format csv -- python3 tools/spmm_bench.py > gpurun_out/pmcsp/p2.log 2>&1 || exit 1
python3 tools/pmc_summary.py "csr_spmm_cols_kernel" gpurun_out/pmcsp > gpurun_out/pmcsp/summary.json
cat gpurun_out/pmcsp/summary.json
