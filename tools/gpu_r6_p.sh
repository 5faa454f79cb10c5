#!/bin/bash
# Round 6: kernel trace of the 20M x 128 north-star UMAP fit (per-kernel time + idle gaps), then
# the same fit untraced for the phase table.
set -o pipefail
mkdir -p gpurun_out/r6p
export TMPDIR=/tmp
OUT=gpurun_out/r6p/trace_umap20M
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/raw -o run -- python3 -u tools/northstar.py --configs umap_cls --warmup 0 --out gpurun_out/r6p/ns_traced.jsonl > gpurun_out/r6p/traced.log 2>&1 || { tail -30 gpurun_out/r6p/traced.log; exit 1; }
python3 tools/trace_summary.py $OUT > gpurun_out/r6p/trace_summary.txt && head -60 gpurun_out/r6p/trace_summary.txt
rm -f $OUT/raw/*/*kernel_trace.csv $OUT/raw/*kernel_trace.csv
timeout -k 10 400 python -u tools/northstar.py --configs umap_cls --warmup 1 --out gpurun_out/r6p/ns_umap.jsonl > gpurun_out/r6p/ns_umap.log 2>&1 || { tail -30 gpurun_out/r6p/ns_umap.log; exit 1; }
cut -c1-1500 gpurun_out/r6p/ns_umap.jsonl
