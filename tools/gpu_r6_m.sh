#!/bin/bash
# Round 6: native Lloyd bookkeeping (large k) — KMeans GPU tests, the KMeans bench, and a
# per-workload glue count of the KMeans fit.
set -o pipefail
mkdir -p gpurun_out/r6m
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_f16_certificate.py -x -q --timeout 200 --timeout-method thread -k "kmeans or certif or f16 or nearest" > gpurun_out/r6m/pytest.log 2>&1 || { tail -40 gpurun_out/r6m/pytest.log; exit 1; }
tail -1 gpurun_out/r6m/pytest.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --algos kmeans --no-transform > gpurun_out/r6m/bench_km.json 2> gpurun_out/r6m/bench_km.err || { tail -20 gpurun_out/r6m/bench_km.err; exit 1; }
python tools/bench_summary.py gpurun_out/r6m/bench_km.json | head -5
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r6m/p_kmeans -o prof --output-format csv -- python3 bench.py --steps 1 --warmup 1 --algos kmeans > gpurun_out/r6m/prof.json 2> gpurun_out/r6m/prof.err || { tail -20 gpurun_out/r6m/prof.err; exit 1; }
python3 tools/glue_summary.py gpurun_out/r6m/p_kmeans kmeans
