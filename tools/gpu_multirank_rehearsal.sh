#!/bin/bash
# Multi-rank rehearsal of the bench on a 1-GPU box: N ranks share cuda:0 over gloo (RCCL refuses
# two ranks per device), exercising every multi-rank device code path except RCCL itself.
set -o pipefail
mkdir -p gpurun_out
for n in ${NS:-2 4}; do
  SRML_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 1 --warmup 1 \
    > gpurun_out/rehearsal_$n.json 2> gpurun_out/rehearsal_$n.err || { echo "n=$n failed"; tail -30 gpurun_out/rehearsal_$n.err; exit 1; }
  python - "$n" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/rehearsal_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("n=" + sys.argv[1], d["ms_per_step"], d["missing_or_failed"] if "missing_or_failed" in d else d["config"].get("missing_or_failed"),
      {k: v["fit_s"] for k, v in d["config"]["workloads"].items()})
PY
done
