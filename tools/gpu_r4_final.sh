#!/bin/bash
# Round-4 end validation on one MI355X: every GPU test, the smoke step, the 1-GPU bench and the
# 125k-row per-rank proxy.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -c 600 gpurun_out/bench_final.json
timeout -k 10 200 python bench.py --rows 125000 > gpurun_out/bench_final_125k.json 2> gpurun_out/bench_final_125k.err || { tail -20 gpurun_out/bench_final_125k.err; exit 1; }
tail -c 300 gpurun_out/bench_final_125k.json
