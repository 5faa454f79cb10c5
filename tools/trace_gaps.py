"""Device busy vs idle in a rocprofv3 kernel trace: the trace is split into bursts at idle gaps
longer than 50 ms (the bench's fits are separated by host work), and per burst the span, the
summed kernel time, the idle time and the largest gaps with the kernels before them are printed."""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:90]))
rows.sort()
bursts, cur = [], [rows[0]]
for r in rows[1:]:
    if r[0] - max(x[1] for x in cur[-50:]) > 50_000_000:
        bursts.append(cur)
        cur = [r]
    else:
        cur.append(r)
bursts.append(cur)
for b in bursts:
    span = (max(x[1] for x in b) - b[0][0]) / 1e6
    if span < 5:
        continue
    busy, end, gaps = 0, b[0][0], []
    for s, e, name in b:
        if s > end:
            gaps.append(((s - end) / 1e6, prev))
        busy += max(0, e - max(s, end))
        end = max(end, e)
        prev = name
    gaps.sort(reverse=True)
    print("burst: %d kernels, span %.2f ms, busy %.2f ms, idle %.2f ms (%d gaps > 20 us)" %
          (len(b), span, busy / 1e6, span - busy / 1e6, sum(1 for g in gaps if g[0] > 0.02)))
    for g, name in gaps[:5]:
        print("   gap %.3f ms after %s" % (g, name))
    if len(b) > 100:  # the in-fit gaps (20 us .. 5 ms) by the kernel before them
        agg = {}
        for g, name in gaps:
            if 0.02 < g < 5.0:
                c, t = agg.get(name, (0, 0.0))
                agg[name] = (c + 1, t + g)
        tot = sum(t for _, t in agg.values())
        print("   in-fit gaps 20 us - 5 ms: %.2f ms over %d gaps" % (tot, sum(c for c, _ in agg.values())))
        for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:8]:
            print("     %7.3f ms  %4d x  after %s" % (t, c, name))
