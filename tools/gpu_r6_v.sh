#!/bin/bash
# Round 6: LDS-DMA staging of the pair search's fp16 item tiles (SRML_KG_DMA=1) — kNN-graph GPU tests
# under it, then 2M / 20M recall + phase A/B against register staging.
set -o pipefail
mkdir -p gpurun_out/r6v
export TMPDIR=/tmp
SRML_KG_DMA=1 timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_umap.py -m gpu -x -q --timeout 200 --timeout-method thread -k "knn or umap or ivf or graph" > gpurun_out/r6v/pytest_dma.log 2>&1 || { tail -40 gpurun_out/r6v/pytest_dma.log; exit 1; }
tail -1 gpurun_out/r6v/pytest_dma.log
for D in 1 0 1 0; do
  SRML_KG_DMA=$D timeout -k 10 300 python -u tools/ivf_recall_sweep.py --rows 20000000 --families classification --nprobe 32 --probe query --queries 500 > gpurun_out/r6v/sweep_20M_dma$D.jsonl 2> gpurun_out/r6v/sweep.err || { tail -20 gpurun_out/r6v/sweep.err; exit 1; }
  echo "DMA=$D"; cut -c1-420 gpurun_out/r6v/sweep_20M_dma$D.jsonl
done
