#!/bin/bash
# GPU tests -> smoke -> 125k-row (per-rank at N=8) bench -> full 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --rows 125000 --steps 2 --warmup 1 > gpurun_out/bench_rows125000.json 2> gpurun_out/bench_rows125000.err || { tail -20 gpurun_out/bench_rows125000.err; exit 1; }
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/bench_rows125000.json", "gpurun_out/bench.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], {k: v["fit_s"] for k, v in d["config"]["workloads"].items()})
PY
