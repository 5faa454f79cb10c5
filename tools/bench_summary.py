"""One line per workload of a bench.py JSON output file: fit seconds, evidence, quality, and the
step summary. python tools/bench_summary.py <bench-output-file>"""
import json
import sys


def main(path: str) -> None:
    line = [x for x in open(path).read().splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    print("value %s ms_per_step %s vs_baseline %s n_gpus %s" % (d["value"], d["ms_per_step"], d["vs_baseline"],
                                                                 d["n_gpus"]))
    for k, w in d["config"]["workloads"].items():
        pr = (w.get("per_rank") or [{}])[0]
        print("%-30s fit %.4f transform %s comm %.4f evidence %s quality %s" % (
            k, w["fit_s"], w.get("transform_s"), pr.get("comm_s", 0.0), w.get("evidence"), w.get("quality")))


if __name__ == "__main__":
    main(sys.argv[1])
