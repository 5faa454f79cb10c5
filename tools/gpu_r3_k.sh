#!/bin/bash
# KMeans checks after a Lloyd-loop change: certified / f16 / delta-sum GPU tests, then the KMeans
# bench rows (random and k-means|| init) at 1M x 3000 and at the 125k-row per-rank shard.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "kmeans or f16 or certified" > gpurun_out/k_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/k_pytest.log; exit 1; }
tail -1 gpurun_out/k_pytest.log
for R in 1000000 125000; do
  timeout -k 10 300 python -u bench.py --rows $R --steps 3 --warmup 1 --algos kmeans,kmeans_init_parallel --no-transform > gpurun_out/k_km_$R.json 2> gpurun_out/k_km_$R.err || { tail -20 gpurun_out/k_km_$R.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/k_km_$R.json').read().strip().splitlines()[-1]);print($R, {k:(v['fit_s'],v['evidence']) for k,v in d['config']['workloads'].items()})"
done
