#!/bin/bash
# fp16 filter LDS-DMA ring A/B: SRML_F16_RING = 10 * (k steps per barrier) + (groups in the ring);
# 0 = default (3 steps x 3 groups). KMeans fit at 1M x 3000, k=1000 + a kernel-only trace per ring.
set -o pipefail
mkdir -p gpurun_out/ring
export TMPDIR=/tmp
for R in 0 23 24 42 18 25 0; do
  SRML_F16_RING=$R timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --algos kmeans --no-transform > gpurun_out/ring/r$R.json 2> gpurun_out/ring/r$R.err || { tail -5 gpurun_out/ring/r$R.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ring/r$R.json').read().strip().splitlines()[-1]);print('ring=$R', d['config']['workloads']['kmeans']['fit_s'])"
done
for R in 0 24 18; do
  SRML_F16_RING=$R timeout -k 10 120 python3 tools/kbench.py --only nearest_f16 > gpurun_out/ring/kb$R.json 2>&1 || exit 1
  echo "ring=$R $(tail -1 gpurun_out/ring/kb$R.json)"
done
