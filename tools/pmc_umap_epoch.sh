#!/bin/bash
# PMC passes over the UMAP epoch kernel (tools/umap_epoch_bench.py, 4M rows).
set -o pipefail
mkdir -p gpurun_out/pmcue
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/umap_epoch_bench.py > gpurun_out/pmcue/plain.log 2>&1 || { tail gpurun_out/pmcue/plain.log; exit 1; }
grep -E "edges|epochs" gpurun_out/pmcue/plain.log
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/pmcue/p1 -o p1 --output-format csv -- python3 tools/umap_epoch_bench.py > gpurun_out/pmcue/p1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum -d gpurun_out/pmcue/p2 -o p2 --output-format csv -- python3 tools/umap_epoch_bench.py > gpurun_out/pmcue/p2.log 2>&1 || exit 1
python3 tools/pmc_summary.py "umap_epoch_kernel" gpurun_out/pmcue > gpurun_out/pmcue/summary.json
cat gpurun_out/pmcue/summary.json
