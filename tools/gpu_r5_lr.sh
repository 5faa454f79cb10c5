#!/bin/bash
# LogReg per-rank proxy (125k rows, the N=8 shard) through the one-rank path and through the
# multi-rank path (SRML_COMM_FORCE_PG=1: a 1-rank RCCL group, per-evaluation all-reduce, captured
# into the QN batch's HIP graph), plus the QN / forced-RCCL GPU tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qn.py tests/test_rccl_forced.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lr_t.log 2>&1 || { tail -30 gpurun_out/lr_t.log; exit 1; }
timeout -k 10 200 python bench.py --rows 125000 --steps 5 --warmup 2 --algos logistic_regression --no-transform > gpurun_out/lr_plain.json 2>gpurun_out/lr_plain.err || exit 1
SRML_COMM_FORCE_PG=1 timeout -k 10 200 python bench.py --rows 125000 --steps 5 --warmup 2 --algos logistic_regression --no-transform > gpurun_out/lr_forced.json 2>gpurun_out/lr_forced.err || { tail -20 gpurun_out/lr_forced.err; exit 1; }
SRML_COMM_FORCE_PG=1 SRML_QN_GRAPH_COMM=0 timeout -k 10 200 python bench.py --rows 125000 --steps 5 --warmup 2 --algos logistic_regression --no-transform > gpurun_out/lr_forced_nograph.json 2>gpurun_out/lr_forced_nograph.err || exit 1
tail -2 gpurun_out/lr_t.log
for f in lr_plain lr_forced lr_forced_nograph; do python3 -c "
import json,sys
l=[x for x in open('gpurun_out/$f.json').read().splitlines() if x.startswith('{')][-1]
w=json.loads(l)['config']['workloads']['logistic_regression']; print('$f', w['fit_s'], w['per_rank'][0]['comm_s'], w['per_rank'][0]['comm_calls'], w['evidence'])"; done
