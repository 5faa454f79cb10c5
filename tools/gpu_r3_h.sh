#!/bin/bash
# fp16 filter tile A/B (256 x 256 one block per CU vs 256 x 128 two blocks per CU) + the 125k-row
# LogisticRegression kernel sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SRML_F16_BN=128 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "f16" > gpurun_out/h_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/h_pytest.log; exit 1; }
tail -1 gpurun_out/h_pytest.log
for bn in 256 128 256 128; do
  SRML_F16_BN=$bn timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --algos kmeans --no-transform > gpurun_out/h_km_$bn.json 2> gpurun_out/h_km_$bn.err || { tail -20 gpurun_out/h_km_$bn.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/h_km_$bn.json').read().strip().splitlines()[-1]);print('bn=$bn', d['config']['workloads']['kmeans']['fit_s'])"
done
bash tools/lr_small_sweep.sh
