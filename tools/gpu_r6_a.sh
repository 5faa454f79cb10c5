#!/bin/bash
# Round-6 first GPU check: the new RF tests (CPU-oracle node split, fused split with sibling
# subtraction), the SPMD-safe persistence in the GPU tier, then the regression-family workloads on
# the make_regression-faithful data (times + held-out R^2) and RFR per-level timings.
set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 400 python -u -m pytest tests/test_rf_levels.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r6a/pytest_rf.log 2>&1 || { tail -40 gpurun_out/r6a/pytest_rf.log; exit 1; }
tail -3 gpurun_out/r6a/pytest_rf.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --algos linear_regression,linear_regression_ridge,linear_regression_elasticnet,random_forest_regressor > gpurun_out/r6a/bench_reg.json 2> gpurun_out/r6a/bench_reg.err || { tail -20 gpurun_out/r6a/bench_reg.err; exit 1; }
python tools/bench_summary.py gpurun_out/r6a/bench_reg.json 2>/dev/null || tail -c 1500 gpurun_out/r6a/bench_reg.json
timeout -k 10 300 python tools/rf_levels.py 1000000 random_forest_regressor > gpurun_out/r6a/rf_levels_rfr.txt 2>&1 || { tail -20 gpurun_out/r6a/rf_levels_rfr.txt; exit 1; }
tail -20 gpurun_out/r6a/rf_levels_rfr.txt
