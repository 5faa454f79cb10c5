#!/bin/bash
# fp16 certified KMeans filter: numerics tests, then the KMeans workloads at 1M rows with a kernel
# trace (bf16 vs f16 filter) and the certified-search unit tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "certified or f16 or split or nearest" > gpurun_out/f16_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/f16_pytest.log; exit 1; }
tail -3 gpurun_out/f16_pytest.log
for mode in bf16 f16; do
  SRML_KMEANS_FILTER=$mode timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --algos kmeans,kmeans_init_parallel --no-transform \
    > gpurun_out/km_$mode.json 2> gpurun_out/km_$mode.err || { echo "bench $mode failed"; tail -30 gpurun_out/km_$mode.err; exit 1; }
  python - $mode <<'PY'
import json, sys
d = json.loads(open("gpurun_out/km_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], {k: (v["fit_s"], v["evidence"]) for k, v in d["config"]["workloads"].items()})
PY
done
cd /tmp && rm -rf $GRAFT_REPO_ROOT/gpurun_out/km_trace && SRML_KMEANS_FILTER=f16 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/km_trace -o km -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --algos kmeans --no-transform > $GRAFT_REPO_ROOT/gpurun_out/km_trace.log 2>&1 || { echo "trace failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/km_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/km_trace -name "*kernel_stats.csv" | head -1)
head -12 "$f" | cut -c1-220
