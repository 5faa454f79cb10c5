#!/bin/bash
# Round 6: rank-insertion merge in the IVF candidate kernels — kNN-graph GPU tests, 2M recall /
# phase sweep (list and query probing), the 20M north-star UMAP fit, and the pair kernel's
# instruction counters.
set -o pipefail
mkdir -p gpurun_out/r6k
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_umap.py -m gpu -x -q --timeout 200 --timeout-method thread -k "knn or umap or ivf or graph" > gpurun_out/r6k/pytest.log 2>&1 || { tail -40 gpurun_out/r6k/pytest.log; exit 1; }
tail -1 gpurun_out/r6k/pytest.log
timeout -k 10 300 python -u tools/ivf_recall_sweep.py --rows 2000000 --families classification,blobs --nprobe 16,32 --probe query > gpurun_out/r6k/sweep_2M.jsonl 2> gpurun_out/r6k/sweep_2M.err || { tail -20 gpurun_out/r6k/sweep_2M.err; exit 1; }
timeout -k 10 300 python -u tools/ivf_recall_sweep.py --rows 2000000 --families classification --nprobe 16,32 --probe list >> gpurun_out/r6k/sweep_2M.jsonl 2>> gpurun_out/r6k/sweep_2M.err || { tail -20 gpurun_out/r6k/sweep_2M.err; exit 1; }
cat gpurun_out/r6k/sweep_2M.jsonl
timeout -k 10 400 python -u tools/northstar.py --configs umap_cls --warmup 1 --out gpurun_out/r6k/ns_umap.jsonl > gpurun_out/r6k/ns_umap.log 2>&1 || { tail -30 gpurun_out/r6k/ns_umap.log; exit 1; }
cut -c1-1400 gpurun_out/r6k/ns_umap.jsonl
timeout -k 10 600 bash tools/pmc_pairs.sh > gpurun_out/r6k/pmc_pairs.log 2>&1 || { tail -20 gpurun_out/r6k/pmc_pairs.log; exit 1; }
tail -30 gpurun_out/r6k/pmc_pairs.log
