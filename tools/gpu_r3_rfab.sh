#!/bin/bash
# RF streamed vs in-memory binning, alternating runs (noise check)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
for mode in 1 0; do
SRML_STREAM_INGEST=$mode timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --algos random_forest_classifier,random_forest_regressor --no-transform > gpurun_out/rfab_$mode$i.json 2> gpurun_out/rfab.err || { tail -20 gpurun_out/rfab.err; exit 1; }
python3 -c "import json,sys;d=json.loads(open('gpurun_out/rfab_$mode$i.json').read().strip().splitlines()[-1]);print('stream=$mode',{k:v['fit_s'] for k,v in d['config']['workloads'].items()})"
done; done
