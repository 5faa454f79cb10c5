#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ring
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "f16 or certified or split" > gpurun_out/ring/pt.log 2>&1 || { tail -30 gpurun_out/ring/pt.log; exit 1; }
tail -1 gpurun_out/ring/pt.log
for R in 0 0 24 25; do
  SRML_F16_RING=$R timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --algos kmeans --no-transform > gpurun_out/ring/s$R.json 2> gpurun_out/ring/s$R.err || { tail -5 gpurun_out/ring/s$R.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ring/s$R.json').read().strip().splitlines()[-1]);print('ring=$R', d['config']['workloads']['kmeans']['fit_s'])"
done
timeout -k 10 120 python3 tools/kbench.py --only nearest_f16 > gpurun_out/ring/kbs.json 2>&1 || exit 1
tail -1 gpurun_out/ring/kbs.json
