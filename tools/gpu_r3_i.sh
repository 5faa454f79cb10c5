#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "f16 or split_rows or certified" > gpurun_out/i_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/i_pytest.log; exit 1; }
tail -1 gpurun_out/i_pytest.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --algos kmeans,kmeans_init_parallel --no-transform > gpurun_out/i_km.json 2> gpurun_out/i_km.err || { tail -20 gpurun_out/i_km.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/i_km.json').read().strip().splitlines()[-1]);print({k:(v['fit_s'],v['evidence']) for k,v in d['config']['workloads'].items()})"
ALGOS=kmeans_init_parallel TAG=kmpar bash tools/gpu_trace_algo.sh | head -30
