"""Timeline of the LAST fit in a rocprofv3 run (kernel trace + roctx marker trace of
``SRML_PROFILE=1``): span, kernel-busy time, idle gaps, per-kernel totals and the tail (what runs
after the last host->device copy), so a fit's fixed costs beyond the H2D can be read off.

    SRML_PROFILE=1 rocprofv3 --kernel-trace --marker-trace --output-format csv -d OUT -o run -- python3 bench.py ...
    python tools/fit_timeline.py OUT [--tail 25]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def _rows(pattern: str):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--tail", type=int, default=25)
    ap.add_argument("--range", default="fit")
    a = ap.parse_args()
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
          for r in _rows(os.path.join(a.out, "**", "*kernel_trace.csv"))]
    ks.sort()
    marks = []
    for r in _rows(os.path.join(a.out, "**", "*marker_api_trace.csv")):
        name = r.get("Message") or r.get("Function") or r.get("Name") or ""
        if name == a.range:
            marks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    marks.sort()
    if marks:
        t0, t1 = marks[-1]
        sel = [k for k in ks if k[0] >= t0 and k[1] <= t1 + 1]
        print("last '%s' range: %.3f ms (host), %d kernels" % (a.range, (t1 - t0) / 1e6, len(sel)))
    else:
        sel = ks[len(ks) // 2:]
        t0 = sel[0][0] if sel else 0
        print("no marker ranges: second half of the dispatches (%d kernels)" % len(sel))
    if not sel:
        return
    span = (sel[-1][1] - sel[0][0]) / 1e6
    busy = 0.0
    last_end = sel[0][0]
    for s, e, _ in sel:
        busy += (e - max(s, last_end)) / 1e6 if e > last_end else 0.0
        last_end = max(last_end, e)
    print("first kernel at +%.3f ms, device span %.3f ms, busy (union) %.3f ms, idle %.3f ms"
          % ((sel[0][0] - t0) / 1e6, span, busy, span - busy))
    tot = defaultdict(lambda: [0, 0.0])
    for s, e, k in sel:
        tot[k][0] += 1
        tot[k][1] += (e - s) / 1e6
    for k, (n, ms) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:20]:
        print("  %9.3f ms %5d  %s" % (ms, n, k[:100]))
    copies = [k for k in sel if "copyBuffer" in k[2]]
    if copies:
        last_copy = max(e for _, e, _ in copies)
        tail = [k for k in sel if k[0] >= last_copy]
        print("after the last copy (+%.3f ms): %d kernels, %.3f ms to the end"
              % ((last_copy - t0) / 1e6, len(tail), (sel[-1][1] - last_copy) / 1e6))
    print("last %d kernels (start offset ms, duration ms):" % a.tail)
    for s, e, k in sel[-a.tail:]:
        print("  +%8.3f %7.3f  %s" % ((s - t0) / 1e6, (e - s) / 1e6, k[:100]))


if __name__ == "__main__":
    main()
