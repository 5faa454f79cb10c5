#!/bin/bash
# A/B of the pair search's item staging at 2M x 128 (per-query probes 32): pre-centred fp16 items
# with two tiles in flight (default) vs the per-tile converting kernel (SRML_IVF_PAIR_H16=0).
set -o pipefail
mkdir -p gpurun_out/r6g
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "knn_pairs or pool_probes or query_probing" > gpurun_out/r6g/pytest.log 2>&1 || { tail -30 gpurun_out/r6g/pytest.log; exit 1; }
tail -1 gpurun_out/r6g/pytest.log
for H in 1 0 1; do
  SRML_IVF_PAIR_H16=$H timeout -k 10 200 python -u tools/ivf_recall_sweep.py --rows 2000000 --families classification --nprobe 32,32 --probe query --queries 300 > gpurun_out/r6g/sweep_h$H.jsonl 2> gpurun_out/r6g/sweep_h$H.err || { tail -20 gpurun_out/r6g/sweep_h$H.err; exit 1; }
  echo "H16=$H $(cat gpurun_out/r6g/sweep_h$H.jsonl)"
done
