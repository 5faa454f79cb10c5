#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_umap_gpu.py tests/test_umap_spectral.py tests/test_ops_gpu.py -k "umap or ivf or knn or spectral or list" -x -q --timeout 200 --timeout-method thread > gpurun_out/u_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/u_pytest.log; exit 1; }
tail -1 gpurun_out/u_pytest.log
OUT=gpurun_out/northstar_umap_r3.jsonl
rm -f $OUT
timeout -k 10 300 python3 -u tools/northstar.py --configs umap --scale 1.0 --out $OUT > gpurun_out/ns_umap2.log 2>&1 || { tail -30 gpurun_out/ns_umap2.log; exit 1; }
cat $OUT
