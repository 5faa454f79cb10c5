#!/bin/bash
# KMeans random-init vs k-means|| fits with the per-phase split (planes / seeding / Lloyd loop)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --algos kmeans,kmeans_init_parallel --no-transform > gpurun_out/kmphase.json 2> gpurun_out/kmphase.err || { tail -20 gpurun_out/kmphase.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/kmphase.json').read().strip().splitlines()[-1]);print({k:(v['fit_s'],v['evidence']) for k,v in d['config']['workloads'].items()})"
