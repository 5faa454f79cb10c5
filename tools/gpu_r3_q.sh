#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "quant or rf_" > gpurun_out/q_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -1 gpurun_out/q_pytest.log
timeout -k 10 120 python3 tools/kbench.py --only quantize > gpurun_out/q_kb.json 2>&1 || { tail -5 gpurun_out/q_kb.json; exit 1; }
tail -1 gpurun_out/q_kb.json
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --algos random_forest_classifier,random_forest_regressor --no-transform > gpurun_out/q_rf.json 2> gpurun_out/q_rf.err || { tail -20 gpurun_out/q_rf.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/q_rf.json').read().strip().splitlines()[-1]);print({k:v['fit_s'] for k,v in d['config']['workloads'].items()})"
