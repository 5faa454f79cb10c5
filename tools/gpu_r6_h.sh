#!/bin/bash
# Round 6: the driver-shaped 1-GPU bench (20 timed steps after 5 warm-up), the 125k-row per-rank
# proxy, a 2-rank gloo rehearsal on the one GPU (multi-rank code paths incl. the fit watchdog and
# the collective empty-shard check), and a kernel-trace --stats of two bench passes (glue count).
set -o pipefail
mkdir -p gpurun_out/r6h
export TMPDIR=/tmp
timeout -k 10 800 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6h/bench_1gpu.json 2> gpurun_out/r6h/bench_1gpu.err || { tail -20 gpurun_out/r6h/bench_1gpu.err; exit 1; }
tail -c 400 gpurun_out/r6h/bench_1gpu.json
timeout -k 10 300 python bench.py --rows 125000 --steps 5 --warmup 2 > gpurun_out/r6h/bench_125k.json 2> gpurun_out/r6h/bench_125k.err || { tail -20 gpurun_out/r6h/bench_125k.err; exit 1; }
tail -c 300 gpurun_out/r6h/bench_125k.json
SRML_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29502 bench.py --gpus 2 --steps 1 --warmup 1 > gpurun_out/r6h/rehearsal_2.json 2> gpurun_out/r6h/rehearsal_2.err || { tail -30 gpurun_out/r6h/rehearsal_2.err; exit 1; }
tail -c 300 gpurun_out/r6h/rehearsal_2.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6h/prof -o prof --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/r6h/prof_bench.json 2> gpurun_out/r6h/prof_bench.err || { tail -20 gpurun_out/r6h/prof_bench.err; exit 1; }
python3 - <<'PY'
import csv, glob
rows = []
for f in glob.glob("gpurun_out/r6h/prof/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
nat = sum(int(r["Calls"]) for r in rows if "at::native" in r["Name"])
print("kernel time %.1f ms, at::native launches %d" % (tot / 1e6, nat))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%9.2f ms %6s  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"], r["Name"][:100]))
for r in sorted((r for r in rows if "at::native" in r["Name"]), key=lambda r: -int(r["Calls"]))[:10]:
    print("%6s calls  %s" % (r["Calls"], r["Name"][:110]))
PY
rm -rf gpurun_out/r6h/prof/*/*kernel_trace.csv
