#!/bin/bash
# PMC of the one-pass fp16 arg-min (srml_nearest_f16_rowloop) in the IVF quantiser / bucketing of a
# 2M x 128 per-query graph: MFMA busy, wave states, LDS traffic, fetch bytes.
set -o pipefail
mkdir -p gpurun_out/pmcr
export TMPDIR=/tmp
P="python3 tools/ivf_recall_sweep.py --rows 2000000 --families classification --nprobe 32 --probe query --queries 100"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/pmcr/p1 -o p1 --output-format csv -- $P > gpurun_out/pmcr/p1.log 2>&1 || { tail -5 gpurun_out/pmcr/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU -d gpurun_out/pmcr/p2 -o p2 --output-format csv -- $P > gpurun_out/pmcr/p2.log 2>&1 || { tail -5 gpurun_out/pmcr/p2.log; exit 1; }
python3 tools/pmc_summary.py nearest_f16_rowloop gpurun_out/pmcr
