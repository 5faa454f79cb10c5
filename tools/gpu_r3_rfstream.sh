#!/bin/bash
# RF binning under the streamed ingest: GPU tests, forest fits streamed vs in-memory binning
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "streamed or rf_ or kmeanspp" > gpurun_out/rfs_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/rfs_pytest.log; exit 1; }
tail -1 gpurun_out/rfs_pytest.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --algos random_forest_classifier,random_forest_regressor --no-transform > gpurun_out/rfs_on.json 2> gpurun_out/rfs_on.err || { tail -20 gpurun_out/rfs_on.err; exit 1; }
SRML_STREAM_INGEST=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --algos random_forest_classifier,random_forest_regressor --no-transform > gpurun_out/rfs_off.json 2> gpurun_out/rfs_off.err || { tail -20 gpurun_out/rfs_off.err; exit 1; }
for f in rfs_on rfs_off; do python3 -c "import json,sys;d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]);print('$f',{k:(v['fit_s'],v['evidence']) for k,v in d['config']['workloads'].items()})"; done
