#!/bin/bash
# Round-5 end validation on one MI355X: every GPU test, the smoke step, the driver-shaped 1-GPU
# bench (20 timed steps after 5 warm-up) and the 125k-row per-rank proxy.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r5_final.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r5_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r5_final.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5_final.log 2>&1 || { tail -20 gpurun_out/smoke_r5_final.log; exit 1; }
tail -1 gpurun_out/smoke_r5_final.log
timeout -k 10 800 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r5_final.json 2> gpurun_out/bench_r5_final.err || { tail -20 gpurun_out/bench_r5_final.err; exit 1; }
tail -c 300 gpurun_out/bench_r5_final.json
timeout -k 10 300 python bench.py --rows 125000 --steps 5 --warmup 2 > gpurun_out/bench_r5_final_125k.json 2> gpurun_out/bench_r5_final_125k.err || { tail -20 gpurun_out/bench_r5_final_125k.err; exit 1; }
tail -c 300 gpurun_out/bench_r5_final_125k.json
