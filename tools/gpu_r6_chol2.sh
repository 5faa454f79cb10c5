#!/bin/bash
# Cholesky trailing update A/B (SRML_POTRF_SYRK 1 = lower-triangle tiles only / 0 = full DGEMM):
# SPD-solve tests under each, then the 125k LinearRegression fit's potrf kernels under rocprof.
set -o pipefail
mkdir -p gpurun_out/chol7
export TMPDIR=/tmp
for V in ${POTRF_SYRKS:-1 0 1 0}; do
  SRML_POTRF_SYRK=$V timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py tests/test_linear_solvers.py -x -q --timeout 120 --timeout-method thread -k "spd or linear or ridge" > gpurun_out/chol7/pytest_$V.log 2>&1 || { tail -30 gpurun_out/chol7/pytest_$V.log; exit 1; }
  echo "V=$V $(tail -1 gpurun_out/chol7/pytest_$V.log)"
  rm -rf gpurun_out/chol7/p_$V
  SRML_POTRF_SYRK=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chol7/p_$V -o p -- python3 bench.py --rows 125000 --steps 2 --warmup 1 --algos linear_regression,linear_regression_ridge --no-transform --no-quality > gpurun_out/chol7/b_$V.json 2> gpurun_out/chol7/b_$V.err || { tail -20 gpurun_out/chol7/b_$V.err; exit 1; }
  python3 - $V <<'PY'
import csv, glob, json, sys
v = sys.argv[1]
d = json.loads(open("gpurun_out/chol7/b_%s.json" % v).read().strip().splitlines()[-1])
print("V=%s" % v, {k: w["fit_s"] for k, w in d["config"]["workloads"].items()})
for r in csv.DictReader(open(glob.glob("gpurun_out/chol7/p_%s/**/*kernel_stats.csv" % v, recursive=True)[0])):
    if "potr" in r["Name"] or "dgemm" in r["Name"]:
        print("   %-40s calls %5s avg %7.1f us total %7.2f ms" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
done
