#!/bin/bash
# Round 6: native RF level bookkeeping + Lloyd bookkeeping + device zero fills — the RF / KMeans GPU
# tests, the full GPU tier, and a per-workload glue count over the eight bench workloads.
set -o pipefail
mkdir -p gpurun_out/r6n
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rf_levels.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6n/pytest_rf.log 2>&1 || { tail -40 gpurun_out/r6n/pytest_rf.log; exit 1; }
tail -1 gpurun_out/r6n/pytest_rf.log
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6n/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6n/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6n/pytest_gpu.log
rm -f gpurun_out/r6n/glue.txt
for A in kmeans pca linear_regression linear_regression_elasticnet linear_regression_ridge logistic_regression random_forest_classifier random_forest_regressor; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r6n/p_$A -o prof --output-format csv -- python3 bench.py --steps 1 --warmup 1 --algos $A > gpurun_out/r6n/$A.json 2> gpurun_out/r6n/$A.err || { tail -20 gpurun_out/r6n/$A.err; exit 1; }
  python3 tools/glue_summary.py gpurun_out/r6n/p_$A $A >> gpurun_out/r6n/glue.txt || exit 1
  rm -f gpurun_out/r6n/p_$A/*kernel_trace.csv
done
grep "==" gpurun_out/r6n/glue.txt
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/r6n/bench.json 2> gpurun_out/r6n/bench.err || { tail -20 gpurun_out/r6n/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r6n/bench.json
