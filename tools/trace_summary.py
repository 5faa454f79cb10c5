"""Summarise a rocprofv3 kernel_trace.csv: per-kernel totals over the timed step (the second
half of the dispatches when warmup == steps) and the per-call durations of selected kernels."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(out_dir: str) -> None:
    files = glob.glob(os.path.join(out_dir, "raw", "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # TRACE_AFTER_GAP_MS: keep only the dispatches after the LAST device-idle gap longer than this
    # (a tool that sleeps between its warm-up and timed runs marks the timed region that way)
    cut_ms = float(os.environ.get("TRACE_AFTER_GAP_MS", "0"))
    if cut_ms > 0 and rows:
        end, cut = rows[0][1], 0
        for j in range(1, len(rows)):
            if (rows[j][0] - end) / 1e6 > cut_ms:
                cut = j
            end = max(end, rows[j][1])
        rows = rows[cut:]
    tot = defaultdict(lambda: [0, 0.0])
    for s, e, k in rows:
        tot[k][0] += 1
        tot[k][1] += (e - s) / 1e6
    span = (rows[-1][1] - rows[0][0]) / 1e6 if rows else 0.0
    print("dispatches %d, first-to-last span %.1f ms (warmup + timed)" % (len(rows), span))
    for k, (n, ms) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:25]:
        print("%9.2f ms %6d  %s" % (ms, n, k[:110]))
    # device-idle analysis: union of kernel intervals vs the span, and the largest gaps (the
    # kernels on either side name where the host was working with nothing in flight)
    busy, cur_s, cur_e, gaps = 0.0, None, None, []
    prev_k = None
    for s, e, k in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1e6
                gaps.append(((s - cur_e) / 1e6, prev_k, k))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_k = k
    if cur_e is not None:
        busy += (cur_e - cur_s) / 1e6
    print("device busy %.1f ms of %.1f ms span (idle %.1f ms)" % (busy, span, span - busy))
    for g, a, b in sorted(gaps, reverse=True)[:int(os.environ.get("TRACE_GAPS", "15"))]:
        print("  gap %8.2f ms after %s -> before %s" % (g, a[:60], b[:60]))
    for pat in ("rf_hist_kernel|rf_hist_wide_kernel", "nearest", "splitmm", "kmeanspp"):
        calls = [(e - s) / 1e6 for s, e, k in rows if any(p in k for p in pat.split("|"))]
        if calls:
            print("%s per call (ms): %s" % (pat, " ".join("%.2f" % c for c in calls[:64])))


if __name__ == "__main__":
    main(sys.argv[1])
