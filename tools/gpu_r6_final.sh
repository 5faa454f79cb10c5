#!/bin/bash
# Round-6 end validation on one MI355X: every GPU test, the smoke step, the driver-shaped 1-GPU
# bench (20 timed steps after 5 warm-up) and the 125k-row per-rank proxy.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r6_final.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r6_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_r6_final.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r6_final.log 2>&1 || { tail -20 gpurun_out/smoke_r6_final.log; exit 1; }
tail -1 gpurun_out/smoke_r6_final.log
timeout -k 10 800 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r6_final.json 2> gpurun_out/bench_r6_final.err || { tail -20 gpurun_out/bench_r6_final.err; exit 1; }
tail -c 300 gpurun_out/bench_r6_final.json
timeout -k 10 300 python bench.py --rows 125000 --steps 5 --warmup 2 > gpurun_out/bench_r6_final_125k.json 2> gpurun_out/bench_r6_final_125k.err || { tail -20 gpurun_out/bench_r6_final_125k.err; exit 1; }
tail -c 300 gpurun_out/bench_r6_final_125k.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6_final -o prof --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_r6_final.json 2> gpurun_out/prof_r6_final.err || { tail -20 gpurun_out/prof_r6_final.err; exit 1; }
python3 tools/glue_summary.py gpurun_out/prof_r6_final all_eight_one_process | head -14
rm -f gpurun_out/prof_r6_final/*kernel_trace.csv
