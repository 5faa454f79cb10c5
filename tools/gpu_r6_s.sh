#!/bin/bash
# Round 6: small-k Lloyd cluster sums as per-lane register adds (n in (32, 64]) — Lloyd GPU tests,
# then the 100M x 64, k = 20 step A/B against the one-hot GEMM sums (SRML_LLOYD_SUMS=mfma).
set -o pipefail
mkdir -p gpurun_out/r6s
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "lloyd or kmeans" > gpurun_out/r6s/pytest.log 2>&1 || { tail -40 gpurun_out/r6s/pytest.log; exit 1; }
tail -1 gpurun_out/r6s/pytest.log
for V in valu mfma valu mfma; do
  SRML_LLOYD_SUMS=$V timeout -k 10 300 python -u tools/lloyd_mfma_bench.py > gpurun_out/r6s/lloyd_$V.json 2> gpurun_out/r6s/lloyd.err || { tail -20 gpurun_out/r6s/lloyd.err; exit 1; }
  echo "SUMS=$V"; tail -c 400 gpurun_out/r6s/lloyd_$V.json
done
