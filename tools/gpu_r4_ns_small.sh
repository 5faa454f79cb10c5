#!/bin/bash
# small-scale checks before the north-star: 2-rank gloo RF (streamed root + reduce-scatter), then a
# kernel trace of the 100M x 64 k=20 KMeans config at 10 % scale (where the Lloyd iteration goes)
set -o pipefail
mkdir -p gpurun_out/nss
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "nearest or cluster_sums or kmeans or lloyd or small" > gpurun_out/nss/pytest_km.log 2>&1 || { tail -40 gpurun_out/nss/pytest_km.log; exit 1; }
tail -1 gpurun_out/nss/pytest_km.log
timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 130 --timeout-method thread > gpurun_out/nss/pytest.log 2>&1 || { tail -40 gpurun_out/nss/pytest.log; exit 1; }
tail -3 gpurun_out/nss/pytest.log
rm -rf gpurun_out/nss/km
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nss/km -o km -- python3 tools/northstar.py --configs kmeans --scale 0.1 --warmup 1 --out gpurun_out/nss/km.jsonl > gpurun_out/nss/km.log 2>&1 || { tail -20 gpurun_out/nss/km.log; exit 1; }
cat gpurun_out/nss/km.jsonl
python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob("gpurun_out/nss/km/**/*kernel_stats.csv", recursive=True)[0])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print("%-70s calls %6s total %9.2f ms avg %8.1f us" % (r["Name"][:70], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
PY
