#!/bin/bash
# Round 6: the whole GPU test tier, then the per-query graph with pre-centred fp16 items at 2M / 20M
# (recall + phase times) and the north-star UMAP 20M classification fit.
set -o pipefail
mkdir -p gpurun_out/r6f
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6f/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r6f/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r6f/pytest_gpu.log
timeout -k 10 300 python -u tools/ivf_recall_sweep.py --rows 2000000 --families classification,blobs --nprobe 16,32 --probe query > gpurun_out/r6f/sweep_2M.jsonl 2> gpurun_out/r6f/sweep_2M.err || { tail -20 gpurun_out/r6f/sweep_2M.err; exit 1; }
cat gpurun_out/r6f/sweep_2M.jsonl
timeout -k 10 400 python -u tools/northstar.py --configs umap_cls --warmup 1 --out gpurun_out/r6f/ns_umap.jsonl > gpurun_out/r6f/ns_umap.log 2>&1 || { tail -30 gpurun_out/r6f/ns_umap.log; exit 1; }
cut -c1-1400 gpurun_out/r6f/ns_umap.jsonl
