#!/bin/bash
# Round-3 check: bootstrap / fp16-filter / RF kernel tests, RF + KMeans bench rows, then the
# north-star UMAP 20M x 128 and LogisticRegression 200M x 256 (chunked generation) at full scale.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "bootstrap or f16 or certified or rf_" > gpurun_out/g_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/g_pytest.log; exit 1; }
tail -1 gpurun_out/g_pytest.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --algos random_forest_classifier,random_forest_regressor,kmeans --no-transform \
  > gpurun_out/g_bench.json 2> gpurun_out/g_bench.err || { echo "bench failed"; tail -30 gpurun_out/g_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/g_bench.json").read().strip().splitlines()[-1])
print({k: (v["fit_s"], v["evidence"]) for k, v in d["config"]["workloads"].items()})
PY
OUT=gpurun_out/northstar_r3c.jsonl
rm -f $OUT
timeout -k 10 300 python3 -u tools/northstar.py --configs umap --scale 1.0 --out $OUT > gpurun_out/ns_umap.log 2>&1 || { tail -30 gpurun_out/ns_umap.log; exit 1; }
cat $OUT
timeout -k 10 600 python3 -u tools/northstar.py --configs logreg --scale 1.0 --out $OUT > gpurun_out/ns_logreg.log 2>&1 || { tail -30 gpurun_out/ns_logreg.log; exit 1; }
tail -1 $OUT
