#!/bin/bash
# streamed-ingest chunk size A/B on the streaming fits (PCA, LinearRegression, forests)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for mb in 96 384 1536 96; do
SRML_INGEST_CHUNK_MB=$mb timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --algos pca,linear_regression,random_forest_classifier,random_forest_regressor --no-transform > gpurun_out/chunk_$mb.json 2> gpurun_out/chunk.err || { tail -20 gpurun_out/chunk.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/chunk_$mb.json').read().strip().splitlines()[-1]);print('$mb MB',{k:(v['fit_s'],v['per_rank'][0]['h2d_s']) for k,v in d['config']['workloads'].items()})"
done
