#!/bin/bash
# Round 6: IVF graph knobs at 20M (quantiser Lloyd iterations, seed-pass list probes): recall and
# phase times, then the north-star UMAP fit (raw_data_ kept from the host rows).
set -o pipefail
mkdir -p gpurun_out/r6r
export TMPDIR=/tmp
for CFG in "10 8" "6 8" "10 5" "6 5"; do
  set -- $CFG
  SRML_IVF_TRAIN_ITERS=$1 SRML_IVF_SEED_PROBES=$2 timeout -k 10 300 python -u tools/ivf_recall_sweep.py --rows 20000000 --families classification --nprobe 32 --probe query --queries 2000 > gpurun_out/r6r/sweep_it$1_sp$2.jsonl 2> gpurun_out/r6r/sweep.err || { tail -20 gpurun_out/r6r/sweep.err; exit 1; }
  echo "iters=$1 seed_probes=$2"; cut -c1-500 gpurun_out/r6r/sweep_it$1_sp$2.jsonl
done
timeout -k 10 400 python -u tools/northstar.py --configs umap_cls --warmup 1 --out gpurun_out/r6r/ns_umap.jsonl > gpurun_out/r6r/ns_umap.log 2>&1 || { tail -30 gpurun_out/r6r/ns_umap.log; exit 1; }
cut -c1-1500 gpurun_out/r6r/ns_umap.jsonl
