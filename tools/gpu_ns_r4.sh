#!/bin/bash
# North-star evidence (one MI355X, round 4). Each config: one warm-up fit, then the timed fit
# (H2D ingest inside it). KMeans 100M x 64 k=20 at tol 0 on uniform rows (all 20 Lloyd
# iterations), RF 50M x 64 data-parallel (held-out accuracy) on one rank and on 2 gloo ranks sharing
# the GPU (reduce-scatter histogram traffic per rank). PART=b: UMAP 20M x 128 (trustworthiness on
# a 20k sample vs a 20k-row fit) and LogReg 200M x 256.
set -o pipefail
mkdir -p gpurun_out
if [ "${PART:-a}" = a ]; then
  timeout -k 10 500 python3 -u tools/northstar.py --configs kmeans,rf --scale 1.0 --warmup 1 --out gpurun_out/northstar_r4_a.jsonl > gpurun_out/ns4_a.log 2>&1 || { tail -30 gpurun_out/ns4_a.log; exit 1; }
  SRML_NS_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/northstar.py --configs rf --scale 1.0 --warmup 1 --out gpurun_out/northstar_r4_b.jsonl > gpurun_out/ns4_b.log 2>&1 || { tail -30 gpurun_out/ns4_b.log; exit 1; }
  cat gpurun_out/northstar_r4_a.jsonl gpurun_out/northstar_r4_b.jsonl
else
  timeout -k 10 900 python3 -u tools/northstar.py --configs umap,logreg --scale 1.0 --warmup 1 --out gpurun_out/northstar_r4_c.jsonl > gpurun_out/ns4_c.log 2>&1 || { tail -30 gpurun_out/ns4_c.log; exit 1; }
  cat gpurun_out/northstar_r4_c.jsonl
fi
