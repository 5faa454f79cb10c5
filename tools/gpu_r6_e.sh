#!/bin/bash
# Round 6: kernel split of the per-query IVF graph build at 2M x 128 (rocprofv3 stats), then the
# counter evidence for the fused RF node split and the LogReg evaluations (tools/pmc_r6.sh).
set -o pipefail
mkdir -p gpurun_out/r6e
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6e/ivf/raw -o ivf --output-format csv -- python3 -u tools/ivf_recall_sweep.py --rows 2000000 --families classification --nprobe 32 --probe query --nnd 0,2 --queries 500 > gpurun_out/r6e/ivf.log 2>&1 || { tail -20 gpurun_out/r6e/ivf.log; exit 1; }
python3 tools/trace_summary.py gpurun_out/r6e/ivf > gpurun_out/r6e/ivf_summary.txt 2>&1; head -30 gpurun_out/r6e/ivf_summary.txt
rm -rf gpurun_out/r6e/ivf/raw
timeout -k 10 400 python -u tools/ivf_recall_sweep.py --rows 20000000 --families classification --nprobe 32 --probe query --nnd 2 --queries 1000 > gpurun_out/r6e/sweep_20M_nnd.jsonl 2> gpurun_out/r6e/sweep_20M_nnd.err || { tail -20 gpurun_out/r6e/sweep_20M_nnd.err; exit 1; }
cat gpurun_out/r6e/sweep_20M_nnd.jsonl
timeout -k 10 900 bash tools/pmc_r6.sh > gpurun_out/r6e/pmc.log 2>&1 || { tail -30 gpurun_out/r6e/pmc.log; exit 1; }
tail -120 gpurun_out/r6e/pmc.log
