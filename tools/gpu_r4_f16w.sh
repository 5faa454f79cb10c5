#!/bin/bash
# (round 4 measurement; the 128 x 128 variant was dropped after it: see profiles/pmc_kmeans_f16_filter_r4_8w_vs_wide.json)
# fp16 certified KMeans filter, 128 x 128 wave tiles (SRML_F16_TILE=wide) vs the 8-wave 128 x 64
# default: certified-search tests under each, kernel time of the filter at 1M x 3000 x 1000, one
# MFMA-busy PMC pass each, then KMeans fit / transform at 1M rows.
set -o pipefail
mkdir -p gpurun_out/f16w
export TMPDIR=/tmp
for T in wide 8w; do
  SRML_F16_TILE=$T timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "certified or f16 or nearest or streamed" > gpurun_out/f16w/pytest_$T.log 2>&1 || { echo "pytest $T failed"; tail -40 gpurun_out/f16w/pytest_$T.log; exit 1; }
  echo "$T: $(tail -1 gpurun_out/f16w/pytest_$T.log)"
done
for T in wide 8w; do
  rm -rf gpurun_out/f16w/k_$T
  SRML_F16_TILE=$T timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f16w/k_$T -o k -- python3 tools/kbench.py --only nearest_f16 > gpurun_out/f16w/k_$T.log 2>&1 || { tail -20 gpurun_out/f16w/k_$T.log; exit 1; }
  python3 - $T <<'PY'
import csv, glob, sys
t = sys.argv[1]
for r in csv.DictReader(open(glob.glob("gpurun_out/f16w/k_%s/**/*kernel_stats.csv" % t, recursive=True)[0])):
    if "glds" in r["Name"] or "select" in r["Name"]:
        print("%-5s %-60s calls %s avg %.1f us min %.1f us" % (t, r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
done
for T in wide 8w; do
  SRML_F16_TILE=$T timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_WAIT_INST_LDS -d gpurun_out/f16w/pmc_$T/p1 -o p1 --output-format csv -- python3 tools/kbench.py --only nearest_f16 --m 250000 > gpurun_out/f16w/pmc_$T.log 2>&1 || exit 1
  SRML_F16_TILE=$T timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/f16w/pmc_$T/p2 -o p2 --output-format csv -- python3 tools/kbench.py --only nearest_f16 --m 250000 > gpurun_out/f16w/pmc2_$T.log 2>&1 || exit 1
  python3 tools/pmc_summary.py "glds_kernel<true, 1," gpurun_out/f16w/pmc_$T > gpurun_out/f16w/pmc_$T.json
  echo "$T pmc: $(cat gpurun_out/f16w/pmc_$T.json | head -c 900)"
done
for T in wide 8w; do
  SRML_F16_TILE=$T timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --algos kmeans --no-quality > gpurun_out/f16w/bench_$T.json 2> gpurun_out/f16w/bench_$T.err || { tail -20 gpurun_out/f16w/bench_$T.err; exit 1; }
  python3 - $T <<'PY'
import json, sys
d = json.loads(open("gpurun_out/f16w/bench_%s.json" % sys.argv[1]).read().strip().splitlines()[-1])
w = d["config"]["workloads"]["kmeans"]
print(sys.argv[1], "kmeans fit %.4f transform %s" % (w["fit_s"], w.get("transform_s")), w["evidence"])
PY
done
