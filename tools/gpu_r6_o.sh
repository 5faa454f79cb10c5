#!/bin/bash
# Round 6: native LSQ statistics / solve glue + segment lower bounds — linear / RF / KMeans GPU tests,
# per-workload glue count (RFC trace kept), and an A/B of the RF level bookkeeping (native vs torch).
set -o pipefail
mkdir -p gpurun_out/r6o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_linear_solvers.py tests/test_rf_levels.py tests/test_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lsq or solve or rf or forest or kmeans or gram or moments or pca or linear" > gpurun_out/r6o/pytest.log 2>&1 || { tail -40 gpurun_out/r6o/pytest.log; exit 1; }
tail -1 gpurun_out/r6o/pytest.log
rm -f gpurun_out/r6o/glue.txt
for A in kmeans pca linear_regression linear_regression_elasticnet linear_regression_ridge logistic_regression random_forest_classifier random_forest_regressor; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r6o/p_$A -o prof --output-format csv -- python3 bench.py --steps 1 --warmup 1 --algos $A > gpurun_out/r6o/$A.json 2> gpurun_out/r6o/$A.err || { tail -20 gpurun_out/r6o/$A.err; exit 1; }
  python3 tools/glue_summary.py gpurun_out/r6o/p_$A $A >> gpurun_out/r6o/glue.txt || exit 1
  if [ "$A" != random_forest_classifier ] && [ "$A" != logistic_regression ]; then rm -f gpurun_out/r6o/p_$A/*kernel_trace.csv; fi
done
grep "==" gpurun_out/r6o/glue.txt
for V in 1 0 1 0; do
  SRML_RF_LEVEL_NATIVE=$V timeout -k 10 300 python bench.py --steps 5 --warmup 1 --algos random_forest_classifier,random_forest_regressor --no-transform --no-quality > gpurun_out/r6o/rf_ab_$V.json 2> gpurun_out/r6o/rf_ab.err || { tail -20 gpurun_out/r6o/rf_ab.err; exit 1; }
  echo "RF_LEVEL_NATIVE=$V"; python tools/bench_summary.py gpurun_out/r6o/rf_ab_$V.json | tail -2 | cut -c1-60
done
