#!/bin/bash
# PMC of the per-query pair search (knn_lists_f16_kernel PAIRS mode) and the list-probing seed at
# 2M x 128 classification rows (per-query probes 32): wave states, LDS, fetch bytes, VALU / MFMA.
set -o pipefail
mkdir -p gpurun_out/pmcp
export TMPDIR=/tmp
P="python3 tools/ivf_recall_sweep.py --rows 2000000 --families classification --nprobe 32 --probe query --queries 100"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcp/t -o t --output-format csv -- $P > gpurun_out/pmcp/t.log 2>&1 || { tail -5 gpurun_out/pmcp/t.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/pmcp/p1 -o p1 --output-format csv -- $P > gpurun_out/pmcp/p1.log 2>&1 || { tail -5 gpurun_out/pmcp/p1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU -d gpurun_out/pmcp/p2 -o p2 --output-format csv -- $P > gpurun_out/pmcp/p2.log 2>&1 || { tail -5 gpurun_out/pmcp/p2.log; exit 1; }
for K in "knn_lists_f16_kernelILb1ELb1E" "knn_lists_f16_kernelILb0E"; do
  echo "== $K"; python3 tools/pmc_summary.py "$K" gpurun_out/pmcp
done
grep -h "knn_lists_f16" gpurun_out/pmcp/t/*/*kernel_stats.csv | cut -c1-200
rm -rf gpurun_out/pmcp/t/*/*kernel_trace.csv
