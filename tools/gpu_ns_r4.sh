#!/bin/bash
# North-star evidence (one MI355X, cold fits incl. H2D), round 4: KMeans 100M x 64 k=20 at tol 0
# (all 20 Lloyd iterations, per-iteration time), RF 50M x 64 data-parallel (held-out accuracy) on
# one rank and on 2 gloo ranks sharing the GPU (reduce-scatter histogram traffic per rank), UMAP
# 20M x 128 (trustworthiness on a 20k sample vs a 20k-row fit), LogReg 200M x 256.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/northstar_r4.jsonl
rm -f $OUT
timeout -k 10 500 python3 -u tools/northstar.py --configs ${CFG_A:-kmeans,rf} --scale 1.0 --out $OUT > gpurun_out/ns4_a.log 2>&1 || { tail -30 gpurun_out/ns4_a.log; exit 1; }
SRML_NS_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/northstar.py --configs rf --scale 1.0 --out $OUT > gpurun_out/ns4_b.log 2>&1 || { tail -30 gpurun_out/ns4_b.log; exit 1; }
timeout -k 10 500 python3 -u tools/northstar.py --configs ${CFG_C:-umap,logreg} --scale 1.0 --out $OUT > gpurun_out/ns4_c.log 2>&1 || { tail -30 gpurun_out/ns4_c.log; exit 1; }
cat $OUT
