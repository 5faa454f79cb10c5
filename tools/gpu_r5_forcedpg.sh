#!/bin/bash
# 125k-row per-rank proxy through the one-rank path and the multi-rank path (SRML_COMM_FORCE_PG=1:
# a 1-rank RCCL group), alternating, all eight workloads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python bench.py --rows 125000 --steps 5 --warmup 2 > gpurun_out/pg_plain_$rep.json 2> gpurun_out/pg_plain_$rep.err || { tail -20 gpurun_out/pg_plain_$rep.err; exit 1; }
  SRML_COMM_FORCE_PG=1 timeout -k 10 300 python bench.py --rows 125000 --steps 5 --warmup 2 > gpurun_out/pg_forced_$rep.json 2> gpurun_out/pg_forced_$rep.err || { tail -20 gpurun_out/pg_forced_$rep.err; exit 1; }
done
for f in gpurun_out/pg_*_?.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1]); w=d['config']['workloads']
print('$f', d['ms_per_step'], d['config'].get('comm_backend'), {k: v['fit_s'] for k, v in w.items()})"; done
