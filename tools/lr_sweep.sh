# logreg loss/grad kernel variant sweep (1M x 3000 fp32): split R D blocks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -k "logreg" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_lr.log 2>&1 || { tail gpurun_out/t_lr.log; exit 1; }
for cfg in ${LR_CFGS:-"2 1 1 2048" "2 1 2 2048" "2 1 3 2048" "2 2 2 2048" "2 1 2 4096" "2 1 3 4096" "2 1 2 1024"}; do
  set -- $cfg
  echo "split=$1 R=$2 D=$3 blocks=$4 $(SRML_LOGREG_SPLIT=$1 SRML_LOGREG_R=$2 SRML_LOGREG_D=$3 SRML_LOGREG_BLOCKS=$4 timeout -k 10 100 python -u tools/kbench.py --only logreg 2>/dev/null | tail -1)" || exit 1
done
