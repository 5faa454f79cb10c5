#!/bin/bash
# IVF quantiser training budget vs graph recall (2M rows) and the 20M UMAP fit / trustworthiness.
set -o pipefail
mkdir -p gpurun_out
for cfg in "10 64" "6 32" "4 32"; do
  set -- $cfg
  SRML_IVF_TRAIN_ITERS=$1 SRML_IVF_TRAIN_ROWS=$2 timeout -k 10 300 python -u tools/ivf_recall_sweep.py --rows 2000000 --nprobe 16,16 --families classification,low_rank > gpurun_out/ivft_$1_$2.jsonl 2>/dev/null || exit 1
  SRML_IVF_TRAIN_ITERS=$1 SRML_IVF_TRAIN_ROWS=$2 timeout -k 10 300 python -u tools/umap_spectral_tol.py --family classification --settings 1e-6:4 > gpurun_out/umapt_$1_$2.jsonl 2>/dev/null || exit 1
  echo "iters=$1 rows=$2"; tail -2 gpurun_out/ivft_$1_$2.jsonl; cat gpurun_out/umapt_$1_$2.jsonl
done
