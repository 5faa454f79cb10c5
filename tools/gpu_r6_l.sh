#!/bin/bash
# Round 6: register-resident query fragments in the IVF candidate kernels; A/B of the per-query
# pair kernel's fp16 item prefetch depth (SRML_KG_H2=1: two register tiles, 0: one) at 2M / 20M.
set -o pipefail
mkdir -p gpurun_out/r6l
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_umap.py -m gpu -x -q --timeout 200 --timeout-method thread -k "knn or umap or ivf or graph" > gpurun_out/r6l/pytest.log 2>&1 || { tail -40 gpurun_out/r6l/pytest.log; exit 1; }
tail -1 gpurun_out/r6l/pytest.log
for H in 1 0; do
  SRML_KG_H2=$H timeout -k 10 300 python -u tools/ivf_recall_sweep.py --rows 2000000 --families classification,blobs --nprobe 32 --probe query > gpurun_out/r6l/sweep_2M_h$H.jsonl 2> gpurun_out/r6l/sweep_2M_h$H.err || { tail -20 gpurun_out/r6l/sweep_2M_h$H.err; exit 1; }
  echo "== H2=$H"; cut -c1-400 gpurun_out/r6l/sweep_2M_h$H.jsonl
done
SRML_KG_H2=0 timeout -k 10 300 python -u tools/ivf_recall_sweep.py --rows 2000000 --families classification --nprobe 16,32 --probe list > gpurun_out/r6l/sweep_2M_list.jsonl 2> gpurun_out/r6l/sweep_2M_list.err || { tail -20 gpurun_out/r6l/sweep_2M_list.err; exit 1; }
cut -c1-400 gpurun_out/r6l/sweep_2M_list.jsonl
for H in 1 0; do
  SRML_KG_H2=$H timeout -k 10 400 python -u tools/ivf_recall_sweep.py --rows 20000000 --families classification --nprobe 32 --probe query --queries 2000 > gpurun_out/r6l/sweep_20M_h$H.jsonl 2> gpurun_out/r6l/sweep_20M_h$H.err || { tail -20 gpurun_out/r6l/sweep_20M_h$H.err; exit 1; }
  echo "== 20M H2=$H"; cut -c1-600 gpurun_out/r6l/sweep_20M_h$H.jsonl
done
