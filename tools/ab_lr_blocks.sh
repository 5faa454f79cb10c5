set -o pipefail
for B in 1024 0 1024 0; do
  SRML_LOGREG_BLOCKS=$B timeout -k 10 200 python -u bench.py --rows 125000 --steps 5 --warmup 2 --algos logistic_regression --no-transform > gpurun_out/ab_$B.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$B.json').read().strip().splitlines()[-1]);print('blocks=$B', d['config']['workloads']['logistic_regression']['fit_s'])"
done
