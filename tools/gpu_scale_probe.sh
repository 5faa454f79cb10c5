#!/bin/bash
# Per-rank work at N=2/4/8 (strong scaling: 1M/N rows) measured on one GPU, plus a rocprofv3
# kernel-stats pass of the full 1M-row suite.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 125000 250000; do
  timeout -k 10 300 python -u bench.py --rows $r --steps 2 --warmup 1 > gpurun_out/bench_rows$r.json 2> gpurun_out/bench_rows$r.err || { tail -20 gpurun_out/bench_rows$r.err; exit 1; }
  echo "rows=$r $(cat gpurun_out/bench_rows$r.json)"
done
bash tools/gpu_prof.sh
