#!/bin/bash
# Round 6: kernel tests touched this round (Lloyd centring, col_moments / xtv accumulation), then
# the north-star UMAP 20M fits (classification + blobs) with per-query probing (fit time,
# trustworthiness, graph recall over all rows), UMAP embedding quality vs graph at 1M, and the
# north-star KMeans (O(k) random init, centred Lloyd loop).
set -o pipefail
mkdir -p gpurun_out/r6d
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_native_paths_gpu.py -x -v --timeout 200 --timeout-method thread -k "lloyd or gram or xtv or moments or scatter or pca or linreg or far_from_origin" > gpurun_out/r6d/pytest.log 2>&1 || { tail -40 gpurun_out/r6d/pytest.log; exit 1; }
tail -2 gpurun_out/r6d/pytest.log
timeout -k 10 600 python -u tools/northstar.py --configs umap_cls,umap --warmup 1 --out gpurun_out/r6d/ns_umap.jsonl > gpurun_out/r6d/ns_umap.log 2>&1 || { tail -30 gpurun_out/r6d/ns_umap.log; exit 1; }
cut -c1-1500 gpurun_out/r6d/ns_umap.jsonl
timeout -k 10 400 python -u tools/umap_graph_quality.py --rows 1000000 --families classification,low_rank --graphs brute,list16,query32 > gpurun_out/r6d/umap_quality_1M.jsonl 2> gpurun_out/r6d/umap_quality_1M.err || { tail -20 gpurun_out/r6d/umap_quality_1M.err; exit 1; }
cat gpurun_out/r6d/umap_quality_1M.jsonl
timeout -k 10 300 python -u tools/northstar.py --configs kmeans --warmup 1 --out gpurun_out/r6d/ns_kmeans.jsonl > gpurun_out/r6d/ns_kmeans.log 2>&1 || { tail -30 gpurun_out/r6d/ns_kmeans.log; exit 1; }
cut -c1-1200 gpurun_out/r6d/ns_kmeans.jsonl
