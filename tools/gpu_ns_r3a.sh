#!/bin/bash
# North-star evidence part A (one MI355X, cold fits incl. H2D): KMeans 100M x 64 and RF 50M x 64
# (data-parallel histograms) at full scale, then RF as 2 ranks sharing the GPU over gloo (the
# per-level histogram all-reduce runs and is timed per rank).
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/northstar_r3.jsonl
rm -f $OUT
timeout -k 10 500 python3 -u tools/northstar.py --configs kmeans,rf --scale 1.0 --out $OUT > gpurun_out/ns_a.log 2>&1 || { tail -30 gpurun_out/ns_a.log; exit 1; }
SRML_NS_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/northstar.py --configs rf --scale 1.0 --out $OUT > gpurun_out/ns_b.log 2>&1 || { tail -30 gpurun_out/ns_b.log; exit 1; }
cat $OUT
