#!/bin/bash
# Round 6: multi-rank rehearsal of the bench after the native bookkeeping changes (2 and 4 gloo
# ranks sharing cuda:0: KMeans device loop all-reduce, RF level kernels, LSQ buffers) + the 2-rank
# UMAP north-star at reduced scale.
set -o pipefail
mkdir -p gpurun_out/r6t
export TMPDIR=/tmp
NS="2 4" timeout -k 10 1000 bash tools/gpu_multirank_rehearsal.sh > gpurun_out/r6t/rehearsal.log 2>&1 || { tail -40 gpurun_out/r6t/rehearsal.log; exit 1; }
cat gpurun_out/r6t/rehearsal.log
cp gpurun_out/rehearsal_2.json gpurun_out/rehearsal_4.json gpurun_out/r6t/
timeout -k 10 500 bash tools/pmc_rowloop.sh > gpurun_out/r6t/pmc_rowloop.log 2>&1 || { tail -20 gpurun_out/r6t/pmc_rowloop.log; exit 1; }
tail -30 gpurun_out/r6t/pmc_rowloop.log
