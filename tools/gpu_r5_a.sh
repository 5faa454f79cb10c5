#!/bin/bash
# Round-5 check A: LogReg per-rank proxy through the multi-rank path (SRML_COMM_FORCE_PG=1) vs the
# one-rank path, UMAP GPU tests, north-star UMAP 20M x 128 (blobs and classification rows) with
# per-phase rows / seconds and the IVF graph's recall vs exact kNN.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --rows 125000 --steps 5 --warmup 2 --algos logistic_regression --no-transform > gpurun_out/lr_plain.json 2>gpurun_out/lr_plain.err || exit 1
SRML_COMM_FORCE_PG=1 timeout -k 10 200 python bench.py --rows 125000 --steps 5 --warmup 2 --algos logistic_regression --no-transform > gpurun_out/lr_forced.json 2>gpurun_out/lr_forced.err || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "umap or spectral" > gpurun_out/umap_gpu_t.log 2>&1 || { tail -30 gpurun_out/umap_gpu_t.log; exit 1; }
timeout -k 10 600 python3 -u tools/northstar.py --configs umap,umap_cls --scale 1.0 --warmup 1 --out gpurun_out/ns_r5_umap.jsonl > gpurun_out/ns_r5_umap.log 2>&1 || { tail -30 gpurun_out/ns_r5_umap.log; exit 1; }
tail -2 gpurun_out/umap_gpu_t.log
cat gpurun_out/ns_r5_umap.jsonl
