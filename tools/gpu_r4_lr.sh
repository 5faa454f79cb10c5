#!/bin/bash
# LogisticRegression evaluation kernel at the per-rank shard (125k x 3000) and at 1M rows:
# grouped-fold epilogue group sizes (SRML_LOGREG_GROUP, 1 = per-block atomics), kernel times
# from rocprofv3 kernel traces; then the LogReg GPU tests.
set -o pipefail
mkdir -p gpurun_out/lr
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "logreg" -x -q --timeout 120 --timeout-method thread > gpurun_out/lr/pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/lr/pytest.log; exit 1; }
tail -1 gpurun_out/lr/pytest.log
for M in 125000 1000000; do
  for G in ${GLIST:-1 4 8 16 32}; do
    rm -rf gpurun_out/lr/p_${M}_$G
    SRML_LOGREG_GROUP=$G timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lr/p_${M}_$G -o p -- python3 tools/kbench.py --only logreg --m $M > gpurun_out/lr/k_${M}_$G.log 2>&1 || { echo "run $M $G failed"; tail -20 gpurun_out/lr/k_${M}_$G.log; exit 1; }
    f=$(find gpurun_out/lr/p_${M}_$G -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$M" "$G" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "logreg_binary_pf" in r["Name"]:
        print("M=%s G=%s calls %s avg %.1f us min %.1f us" % (sys.argv[2], sys.argv[3], r["Calls"],
              float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
  done
done
