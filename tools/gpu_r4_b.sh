#!/bin/bash
# Round-4 LogReg iteration + per-workload timelines at the 125k shard:
#   tests of the evaluation / QN kernels; kernel times of the evaluation (+ fold) and of the QN step
#   (single-block vs four multi-block launches vs one fused launch that also folds the evaluation); 125k
#   LogReg bench; then tools/gpu_r4_trace.sh (timelines of every workload's timed fit).
set -o pipefail
mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_qn.py -k "logreg or qn or logistic" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/pytest.log 2>&1 || { tail -30 gpurun_out/r4b/pytest.log; exit 1; }
tail -1 gpurun_out/r4b/pytest.log
rm -rf gpurun_out/r4b/p
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b/p -o p -- python3 tools/kbench.py --only logreg --m 125000 > gpurun_out/r4b/k.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for r in csv.DictReader(open(glob.glob("gpurun_out/r4b/p/**/*kernel_stats.csv", recursive=True)[0])):
    if "logreg" in r["Name"] or "fold" in r["Name"]:
        print("%-40s calls %s avg %.1f us min %.1f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
for MB in single mb fused; do
  rm -rf gpurun_out/r4b/lr_$MB
  SRML_QN_STEP=$MB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b/lr_$MB -o p -- python3 bench.py --rows 125000 --steps 2 --warmup 1 --algos logistic_regression --no-transform --no-quality > gpurun_out/r4b/lr_$MB.json 2> gpurun_out/r4b/lr_$MB.err || { tail -20 gpurun_out/r4b/lr_$MB.err; exit 1; }
  python3 - $MB <<'PY'
import csv, glob, json, sys
mb = sys.argv[1]
d = json.loads(open("gpurun_out/r4b/lr_%s.json" % mb).read().strip().splitlines()[-1])
w = d["config"]["workloads"]["logistic_regression"]
print("QN_STEP=%s logreg 125k fit %.4f s (under rocprof) evals %s" % (mb, w["fit_s"], w["evidence"].get("n_evals")))
for r in csv.DictReader(open(glob.glob("gpurun_out/r4b/lr_%s/**/*kernel_stats.csv" % mb, recursive=True)[0])):
    if "qn_" in r["Name"] or "logreg" in r["Name"] or "fold" in r["Name"]:
        print("   %-36s calls %s avg %.1f us" % (r["Name"][:36], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
[ -n "$TRACE" ] && bash tools/gpu_r4_trace.sh
true
