#!/bin/bash
# Small-k Lloyd label book (delta steps): the kernel / loop tests, then the 100M x 64 k = 20
# north-star fit with delta steps on and off (alternating).
set -o pipefail
mkdir -p gpurun_out/r6w
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "lloyd or kmeans" > gpurun_out/r6w/pytest.log 2>&1 || { tail -40 gpurun_out/r6w/pytest.log; exit 1; }
tail -2 gpurun_out/r6w/pytest.log
for d in 1 0 1 0; do
  SRML_LLOYD_SMALL_DELTA=$d timeout -k 10 300 python -u tools/northstar.py --configs kmeans --warmup 1 --out gpurun_out/r6w/ns_kmeans_delta$d.jsonl > gpurun_out/r6w/ns_$d.log 2>&1 || { tail -30 gpurun_out/r6w/ns_$d.log; exit 1; }
  echo "delta=$d $(tail -1 gpurun_out/r6w/ns_kmeans_delta$d.jsonl | cut -c1-150) $(tail -1 gpurun_out/r6w/ns_kmeans_delta$d.jsonl | grep -o '"phase_s.*')"
done
