#!/bin/bash
# register-resident vector cand_exact: GPU tests, KMeans A/B, trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SRML_CAND_EXACT=1 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "f16 or gather or certified or kmeans" > gpurun_out/ce_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/ce_pytest.log; exit 1; }
tail -1 gpurun_out/ce_pytest.log
for mode in 1 0 1; do
SRML_CAND_EXACT=$mode timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --algos kmeans,kmeans_init_parallel --no-transform > gpurun_out/ce_$mode.json 2> gpurun_out/ce.err || { tail -20 gpurun_out/ce.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/ce_$mode.json').read().strip().splitlines()[-1]);print('vec=$mode',{k:(v['fit_s'],v['evidence'].get('phase_s')) for k,v in d['config']['workloads'].items()})"
done
SRML_CAND_EXACT=1 ALGOS=kmeans TAG=km_ce bash tools/gpu_trace_algo.sh | head -10
