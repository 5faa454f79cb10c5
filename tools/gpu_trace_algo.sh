#!/bin/bash
# Per-dispatch kernel trace of one fit of the given workloads (ALGOS), summarised per kernel
# and, for the RF histogram, per call (= per tree level). Output under gpurun_out/trace_<tag>/.
set -o pipefail
ALGOS=${ALGOS:-random_forest_regressor}
TAG=${TAG:-$ALGOS}
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/raw -o run -- python3 -u bench.py --steps 1 --warmup 1 --algos $ALGOS --no-transform $BENCH_EXTRA > $OUT/bench.json 2> $OUT/bench.err || { echo "trace failed"; tail -30 $OUT/bench.err; exit 1; }
python3 tools/trace_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
