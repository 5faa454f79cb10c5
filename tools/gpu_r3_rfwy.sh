#!/bin/bash
# fused (weight, label) packing per tree level: GPU tests, forest fits, RFC trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "streamed or rf_ or forest" > gpurun_out/rfwy_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/rfwy_pytest.log; exit 1; }
tail -1 gpurun_out/rfwy_pytest.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --algos random_forest_classifier,random_forest_regressor --no-transform > gpurun_out/rfwy_$i.json 2> gpurun_out/rfwy.err || { tail -20 gpurun_out/rfwy.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/rfwy_$i.json').read().strip().splitlines()[-1]);print({k:(v['fit_s'],v['evidence']) for k,v in d['config']['workloads'].items()})"
done
ALGOS=random_forest_classifier TAG=rfc_wy bash tools/gpu_trace_algo.sh | head -24
