#!/bin/bash
# Small-k Lloyd label book, tile-skipping delta steps: per-iteration diag (the loop's rule, full
# steps counting moved rows, no book)
set -o pipefail
mkdir -p gpurun_out/r6x
for v in "" "--nobook"; do
timeout -k 10 200 python -u tools/lloyd_delta_diag.py $v > gpurun_out/r6x/d$v.jsonl 2> gpurun_out/r6x/d.err || { tail -20 gpurun_out/r6x/d.err; exit 1; }
echo "diag $v"; cut -c1-100 gpurun_out/r6x/d$v.jsonl
done
