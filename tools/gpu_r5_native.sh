#!/bin/bash
# Round-5 native-path check: kernel trace of the item-8 configs, then the library-kernel check.
set -o pipefail
mkdir -p gpurun_out/np5
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/np5/raw -o np -- python3 tools/native_paths.py --set r5 > gpurun_out/np5/log.txt 2>&1 || { tail -30 gpurun_out/np5/log.txt; exit 1; }
f=$(find gpurun_out/np5/raw -name "np_kernel_stats.csv" | head -1)
cp "$f" gpurun_out/np5/kernel_stats.csv
python3 tools/native_paths.py --set r5 --check gpurun_out/np5/kernel_stats.csv > gpurun_out/np5/check.txt 2>&1; rc=$?
rm -rf gpurun_out/np5/raw
cat gpurun_out/np5/log.txt | grep -v amdgpu.ids; cat gpurun_out/np5/check.txt
exit $rc
