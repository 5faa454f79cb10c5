#!/bin/bash
# RF classifier at the headline shape on the reference-faithful data: host profile of one fit,
# then a kernel + roctx timeline of a bench step (idle gaps, per-kernel totals).
set -o pipefail
mkdir -p gpurun_out/rf5
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/suite_host_profile.py 1000000 random_forest_classifier > gpurun_out/rf5/host.txt 2>&1 || { tail -20 gpurun_out/rf5/host.txt; exit 1; }
SRML_PROFILE=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/rf5/raw -o run -- python3 bench.py --steps 1 --warmup 1 --algos random_forest_classifier --no-transform --no-quality > gpurun_out/rf5/bench.json 2> gpurun_out/rf5/bench.err || { tail -20 gpurun_out/rf5/bench.err; exit 1; }
python3 tools/fit_timeline.py gpurun_out/rf5/raw > gpurun_out/rf5/timeline.txt 2>&1
rm -rf gpurun_out/rf5/raw
cat gpurun_out/rf5/host.txt | head -40
head -60 gpurun_out/rf5/timeline.txt
