#!/bin/bash
# Round 6: KMeans tests after the fused centre prep, KMeans bench (1M and 125k), the pair-search
# PMC, and a kernel-trace glue count of the KMeans + PCA / LinReg fits.
set -o pipefail
mkdir -p gpurun_out/r6i
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_f16_certificate.py -x -q --timeout 200 --timeout-method thread -k "certif or f16 or kmeans or nearest or gram or moments" > gpurun_out/r6i/pytest.log 2>&1 || { tail -30 gpurun_out/r6i/pytest.log; exit 1; }
tail -1 gpurun_out/r6i/pytest.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --algos kmeans,pca,linear_regression --no-transform > gpurun_out/r6i/bench_km.json 2> gpurun_out/r6i/bench_km.err || { tail -20 gpurun_out/r6i/bench_km.err; exit 1; }
python tools/bench_summary.py gpurun_out/r6i/bench_km.json | head -5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6i/prof -o prof --output-format csv -- python3 bench.py --steps 1 --warmup 1 --algos kmeans,pca,linear_regression > gpurun_out/r6i/prof.json 2> gpurun_out/r6i/prof.err || { tail -20 gpurun_out/r6i/prof.err; exit 1; }
python3 - <<'PY'
import csv, glob
rows = []
for f in glob.glob("gpurun_out/r6i/prof/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
nat = sum(int(r["Calls"]) for r in rows if "at::native" in r["Name"])
print("at::native launches (kmeans + pca + linreg, two passes incl. transforms): %d" % nat)
for r in sorted((r for r in rows if "at::native" in r["Name"]), key=lambda r: -int(r["Calls"]))[:8]:
    print("%6s calls  %s" % (r["Calls"], r["Name"][:110]))
PY
rm -rf gpurun_out/r6i/prof/*/*kernel_trace.csv
timeout -k 10 700 bash tools/pmc_pairs.sh > gpurun_out/r6i/pmc_pairs.log 2>&1 || { tail -20 gpurun_out/r6i/pmc_pairs.log; exit 1; }
tail -60 gpurun_out/r6i/pmc_pairs.log
