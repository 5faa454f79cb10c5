#!/bin/bash
# Round-4 iteration: GPU tests of the touched kernels, the LogReg evaluation with / without the
# partial-row fold (kernel times from rocprofv3), then the 125k-row LogReg + suite bench.
set -o pipefail
mkdir -p gpurun_out/r4a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_ops_gpu.py tests/test_metrics_partials.py tests/test_sparse.py tests/test_umap_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a/pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/r4a/pytest.log; exit 1; }
tail -1 gpurun_out/r4a/pytest.log
for M in 125000 1000000; do
  for F in 0 1; do
    rm -rf gpurun_out/r4a/p_${M}_$F
    SRML_LOGREG_FOLD=$F timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4a/p_${M}_$F -o p -- python3 tools/kbench.py --only logreg --m $M > gpurun_out/r4a/k_${M}_$F.log 2>&1 || { echo "run $M $F failed"; tail -20 gpurun_out/r4a/k_${M}_$F.log; exit 1; }
    f=$(find gpurun_out/r4a/p_${M}_$F -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$M" "$F" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "logreg_binary_pf" in r["Name"] or "fold_rows" in r["Name"]:
        print("M=%s FOLD=%s %-28s calls %s avg %.1f us min %.1f us" % (sys.argv[2], sys.argv[3], r["Name"][:28], r["Calls"],
              float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
  done
done
timeout -k 10 300 python -u bench.py --rows 125000 --steps 2 --warmup 1 --algos ${ALGOS:-logistic_regression} --no-transform > gpurun_out/r4a/bench125k.json 2> gpurun_out/r4a/bench125k.err || { tail -20 gpurun_out/r4a/bench125k.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r4a/bench125k.json").read().strip().splitlines()[-1])
for k, v in d["config"]["workloads"].items():
    print("125k %-28s fit %.4f s  per_rank %s  ev %s" % (k, v["fit_s"], v["per_rank"], v["evidence"]))
PY
