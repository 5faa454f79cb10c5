#!/bin/bash
# register-resident k-means++ kernel: GPU tests, A/B against the chunked block kernel, k-means|| fit
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "kmeanspp" > gpurun_out/kpp_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/kpp_pytest.log; exit 1; }
tail -1 gpurun_out/kpp_pytest.log
timeout -k 10 200 python -u tools/kbench.py --m 1000 --n 64 --only kpp > gpurun_out/kpp_reg.json 2>&1 && tail -1 gpurun_out/kpp_reg.json || exit 1
SRML_KPP_KERNEL=block timeout -k 10 200 python -u tools/kbench.py --m 1000 --n 64 --only kpp > gpurun_out/kpp_block.json 2>&1 && tail -1 gpurun_out/kpp_block.json || exit 1
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --algos kmeans,kmeans_init_parallel --no-transform > gpurun_out/kpp_km.json 2> gpurun_out/kpp_km.err || { tail -20 gpurun_out/kpp_km.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/kpp_km.json').read().strip().splitlines()[-1]);print({k:(v['fit_s'],v['evidence']) for k,v in d['config']['workloads'].items()})"
ALGOS=kmeans_init_parallel TAG=kmpar_kpp bash tools/gpu_trace_algo.sh | head -30
