#!/bin/bash
# Per-query IVF probing: kernel tests, then graph recall / time at 2M (three families, list vs
# query probing) and 20M classification rows.
set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 200 --timeout-method thread -k "knn_pairs or pool_probes or query_probing or knn_graph_ivf_f16 or knn_lists_f16" > gpurun_out/r6b/pytest.log 2>&1 || { tail -40 gpurun_out/r6b/pytest.log; exit 1; }
tail -3 gpurun_out/r6b/pytest.log
timeout -k 10 400 python -u tools/ivf_recall_sweep.py --rows 2000000 --families classification,low_rank,blobs --nprobe 16,32 > gpurun_out/r6b/sweep_2M.jsonl 2> gpurun_out/r6b/sweep_2M.err || { tail -20 gpurun_out/r6b/sweep_2M.err; exit 1; }
cat gpurun_out/r6b/sweep_2M.jsonl
timeout -k 10 400 python -u tools/ivf_recall_sweep.py --rows 20000000 --families classification --nprobe 16,32 --probe query --queries 1000 > gpurun_out/r6b/sweep_20M.jsonl 2> gpurun_out/r6b/sweep_20M.err || { tail -20 gpurun_out/r6b/sweep_20M.err; exit 1; }
cat gpurun_out/r6b/sweep_20M.jsonl
