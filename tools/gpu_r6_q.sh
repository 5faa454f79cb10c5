#!/bin/bash
# Round 6: one-pass fp16 arg-min for IVF bucketing / quantiser labels — its GPU test, the kNN / UMAP
# GPU tests, the 2M recall sweep and the 20M north-star UMAP fit.
set -o pipefail
mkdir -p gpurun_out/r6q
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "rowloop" > gpurun_out/r6q/pytest_rowloop.log 2>&1 || { tail -40 gpurun_out/r6q/pytest_rowloop.log; exit 1; }
tail -1 gpurun_out/r6q/pytest_rowloop.log
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_umap.py -m gpu -x -q --timeout 200 --timeout-method thread -k "knn or umap or ivf or graph or quantiz or nearest" > gpurun_out/r6q/pytest.log 2>&1 || { tail -40 gpurun_out/r6q/pytest.log; exit 1; }
tail -1 gpurun_out/r6q/pytest.log
timeout -k 10 300 python -u tools/ivf_recall_sweep.py --rows 2000000 --families classification,blobs --nprobe 32 --probe query > gpurun_out/r6q/sweep_2M.jsonl 2> gpurun_out/r6q/sweep_2M.err || { tail -20 gpurun_out/r6q/sweep_2M.err; exit 1; }
cut -c1-400 gpurun_out/r6q/sweep_2M.jsonl
timeout -k 10 400 python -u tools/northstar.py --configs umap_cls --warmup 1 --out gpurun_out/r6q/ns_umap.jsonl > gpurun_out/r6q/ns_umap.log 2>&1 || { tail -30 gpurun_out/r6q/ns_umap.log; exit 1; }
cut -c1-1500 gpurun_out/r6q/ns_umap.jsonl
