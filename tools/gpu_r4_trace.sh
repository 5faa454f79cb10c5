#!/bin/bash
# Per-workload timeline of the timed fit at a given row count (default the 125k per-rank shard of
# an 8-GPU fit): kernel + roctx marker traces, summarised by tools/fit_timeline.py.
set -o pipefail
ROWS=${ROWS:-125000}
OUT=gpurun_out/tl_$ROWS
mkdir -p $OUT
export TMPDIR=/tmp
for A in ${ALGOS:-kmeans pca linear_regression linear_regression_elasticnet linear_regression_ridge logistic_regression random_forest_classifier random_forest_regressor}; do
  rm -rf $OUT/$A
  SRML_PROFILE=1 timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $OUT/$A -o run -- python3 -u bench.py --rows $ROWS --steps 1 --warmup 1 --algos $A --no-transform --no-quality > $OUT/$A.json 2> $OUT/$A.err || { echo "trace $A failed"; tail -20 $OUT/$A.err; exit 1; }
  echo "=== $A"
  python3 tools/fit_timeline.py $OUT/$A --tail ${TAIL:-20} | tee $OUT/$A.timeline.txt
done
