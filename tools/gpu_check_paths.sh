#!/bin/bash
# fp64-path library-kernel check + RF transform timing (one GPU call).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -k "rf_predict" -x -q --timeout 120 --timeout-method thread > gpurun_out/cp_pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/cp_pytest.log; exit 1; }
tail -1 gpurun_out/cp_pytest.log
rm -rf gpurun_out/fp64
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp64 -o fp64 -- python3 tools/fp64_paths.py > gpurun_out/fp64.log 2>&1 \
  || { echo "fp64 run failed"; tail -30 gpurun_out/fp64.log; exit 1; }
grep -v "^W\|warn" gpurun_out/fp64.log | tail -8
f=$(find gpurun_out/fp64 -name "*kernel_stats.csv" | head -1)
python tools/fp64_paths.py --check "$f" || true
timeout -k 10 600 python -u bench.py --rows 1000000 --steps 1 --warmup 1 --algos random_forest_classifier,random_forest_regressor,pca,logistic_regression > gpurun_out/cp_bench.json 2> gpurun_out/cp_bench.err \
  || { echo "bench failed"; tail -30 gpurun_out/cp_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/cp_bench.json").read().strip().splitlines()[-1])
for k, v in d["config"]["workloads"].items():
    print("  %-26s fit %.4f s  transform %s  %s" % (k, v["fit_s"], v.get("transform_s"), v.get("transform_error", "")))
PY
