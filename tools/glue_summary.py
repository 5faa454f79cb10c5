"""Summarise the torch-library launches (at::native, rocprim) of one rocprofv3 --stats run.

Usage: python tools/glue_summary.py <rocprof output dir> <tag>
"""
import csv
import glob
import sys


def main():
    d, tag = sys.argv[1], sys.argv[2]
    rows = []
    for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    glue = [r for r in rows if "at::native" in r["Name"] or "rocprim" in r["Name"]]
    own = [r for r in rows if r not in glue]
    n_glue = sum(int(r["Calls"]) for r in glue)
    n_own = sum(int(r["Calls"]) for r in own)
    t_glue = sum(int(r["TotalDurationNs"]) for r in glue) / 1e6
    print("== %s: glue launches %d (%.2f ms), own kernels %d" % (tag, n_glue, t_glue, n_own))
    for r in sorted(glue, key=lambda r: -int(r["Calls"]))[:12]:
        print("%6s  %s" % (r["Calls"], r["Name"][:140]))


if __name__ == "__main__":
    main()
