#!/bin/bash
# North-star evidence part B: UMAP 20M x 128 at full scale, LogisticRegression at 0.75
# (150M x 256, 154 GB pinned host shard); then PMC passes over the certified KMeans pass.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/northstar_r3b.jsonl
rm -f $OUT
timeout -k 10 500 python3 -u tools/northstar.py --configs umap --scale 1.0 --out $OUT > gpurun_out/ns_c.log 2>&1 || { tail -30 gpurun_out/ns_c.log; exit 1; }
timeout -k 10 500 python3 -u tools/northstar.py --configs logreg --scale 0.75 --out $OUT > gpurun_out/ns_d.log 2>&1 || { tail -30 gpurun_out/ns_d.log; exit 1; }
cat $OUT
bash tools/pmc_certified.sh
