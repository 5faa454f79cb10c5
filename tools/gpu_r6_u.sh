#!/bin/bash
# Round 6: spectral-init Ritz tolerance (umap-learn's eigsh uses 1e-4) — 20M north-star UMAP fit
# and trustworthiness at 1e-4 / 1e-5 vs the 1e-6 default.
set -o pipefail
mkdir -p gpurun_out/r6u
export TMPDIR=/tmp
for T in 1e-4 1e-5; do
  SRML_UMAP_SPECTRAL_TOL=$T timeout -k 10 400 python -u tools/northstar.py --configs umap_cls --warmup 1 --out gpurun_out/r6u/ns_umap_tol$T.jsonl > gpurun_out/r6u/ns_$T.log 2>&1 || { tail -30 gpurun_out/r6u/ns_$T.log; exit 1; }
  echo "tol=$T"; cut -c1-1500 gpurun_out/r6u/ns_umap_tol$T.jsonl
done
