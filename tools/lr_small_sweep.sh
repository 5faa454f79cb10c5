#!/bin/bash
# LogisticRegression loss/grad kernel at the per-rank shard of an 8-GPU fit (125k x 3000): grid
# size / rows-per-batch / prefetch-depth sweep (each setting is read once per process).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/lr_small_sweep.txt
: > $out
for B in 0 512 768 1536; do
  for RD in "1 3" "2 2" "1 2"; do
    set -- $RD
    r=$(SRML_LOGREG_BLOCKS=$B SRML_LOGREG_R=$1 SRML_LOGREG_D=$2 timeout -k 5 60 python3 tools/kbench.py --only logreg --m ${M:-125000} 2>/dev/null | tail -1) || exit 1
    echo "blocks=$B R=$1 D=$2 $r" | tee -a $out
  done
done
