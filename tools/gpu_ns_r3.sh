#!/bin/bash
# North-star evidence, one MI355X (BASELINE.json configs; one cold fit each incl. H2D):
# KMeans 100M x 64 and RF 50M x 64 (data-parallel histograms) and UMAP 20M x 128 at full scale,
# RF again as 2 ranks sharing the GPU over gloo (the per-level histogram all-reduce runs and is
# timed per rank), LogisticRegression at 0.75 (150M x 256, 154 GB pinned host shard).
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/northstar_r3.jsonl
rm -f $OUT
timeout -k 10 400 python3 -u tools/northstar.py --configs kmeans,rf --scale 1.0 --out $OUT > gpurun_out/ns_a.log 2>&1 || { tail -30 gpurun_out/ns_a.log; exit 1; }
SRML_NS_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/northstar.py --configs rf --scale 1.0 --out $OUT > gpurun_out/ns_b.log 2>&1 || { tail -30 gpurun_out/ns_b.log; exit 1; }
timeout -k 10 500 python3 -u tools/northstar.py --configs umap --scale 1.0 --out $OUT > gpurun_out/ns_c.log 2>&1 || { tail -30 gpurun_out/ns_c.log; exit 1; }
timeout -k 10 500 python3 -u tools/northstar.py --configs logreg --scale 0.75 --out $OUT > gpurun_out/ns_d.log 2>&1 || { tail -30 gpurun_out/ns_d.log; exit 1; }
cat $OUT
