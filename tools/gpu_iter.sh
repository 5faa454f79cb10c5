#!/bin/bash
# One GPU iteration: selected tests -> selected bench workloads (1M rows and the 125k-row per-rank
# proxy). Env: TESTS (pytest args, default tests -m gpu), ALGOS (bench --algos, default all),
# STEPS (default 2), ROWS_LIST (default "1000000 125000"), PROF=1 adds a rocprofv3 kernel-stats run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests -m gpu"}
ALGOS=${ALGOS:-all}
STEPS=${STEPS:-2}
ROWS_LIST=${ROWS_LIST:-"1000000 125000"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/it_pytest.log 2>&1 \
    || { echo "pytest failed"; tail -60 gpurun_out/it_pytest.log; exit 1; }
  tail -2 gpurun_out/it_pytest.log
fi
for R in $ROWS_LIST; do
  timeout -k 10 600 python -u bench.py --rows $R --steps $STEPS --warmup 1 --algos $ALGOS > gpurun_out/it_bench_$R.json 2> gpurun_out/it_bench_$R.err \
    || { echo "bench $R failed"; tail -30 gpurun_out/it_bench_$R.err; exit 1; }
  python - "$R" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/it_bench_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("rows", sys.argv[1], "ms/step", d["ms_per_step"], "failed", d["config"]["missing_or_failed"])
for k, v in d["config"]["workloads"].items():
    print("  %-30s %.4f s  %s" % (k, v["fit_s"], {a: b for a, b in v.items() if a not in ("fit_s", "speedup_vs_spark_cpu", "ref_gpu_fit_s", "vs_ref_gpu")}))
PY
done
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o it -- python3 bench.py --rows ${PROF_ROWS:-1000000} --steps 1 --warmup 1 --algos $ALGOS > gpurun_out/it_prof.log 2>&1 \
    || { echo "rocprof failed"; tail -30 gpurun_out/it_prof.log; exit 1; }
  f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
  python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:25]:
    print("%6.2f%% %10.3f ms %6s  %s" % (100 * float(r["TotalDurationNs"]) / tot, float(r["TotalDurationNs"]) / 1e6, r["Calls"], r["Name"][:110]))
PY
fi
