"""Summarise tools/pmc_r6.sh: per kernel family, dispatches, kernel time (kernel trace), PMC sums,
and derived ratios (HBM bytes / kernel time, MFMA-free LDS conflict fraction, wave-state split)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

GROUPS = {
    "random_forest_classifier": {"rf_node_split": "rf_node_split_kernel", "rf_hist_wide": "rf_hist_wide_kernel",
                                 "rf_hist": "rf_hist_kernel<"},
    "logistic_regression": {"logreg_evaluations": "logreg_binary", "qn_step": "qn_"},
}


def _times(d):
    out = defaultdict(lambda: [0, 0.0])
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[r["Kernel_Name"]][0] += 1
            out[r["Kernel_Name"]][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return out


def _pmc(d, pat):
    tot = defaultdict(float)
    disp = set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat not in r.get("Kernel_Name", ""):
                continue
            disp.add((f, r.get("Dispatch_Id")))
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    return tot, len(disp)


def main(root):
    res = {}
    for w, groups in GROUPS.items():
        base = os.path.join(root, w)
        if not os.path.isdir(base):
            continue
        times = _times(os.path.join(base, "t"))
        for g, pat in groups.items():
            n = sum(v[0] for k, v in times.items() if pat in k)
            ms = sum(v[1] for k, v in times.items() if pat in k)
            if n == 0:
                continue
            p1, d1 = _pmc(os.path.join(base, "p1"), pat)
            p2, d2 = _pmc(os.path.join(base, "p2"), pat)
            rec = {"kernels": sorted({k[:90] for k in times if pat in k}), "dispatches": n, "kernel_ms": round(ms, 3)}
            rec.update({k: v for k, v in sorted({**p1, **p2}.items())})
            wc = p1.get("SQ_WAVE_CYCLES", 0.0)
            if wc:
                rec["wait_any_frac"] = round(p1.get("SQ_WAIT_ANY", 0) / wc, 4)
                rec["wait_inst_any_frac"] = round(p1.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
                rec["active_inst_frac"] = round(p1.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
            if p1.get("SQ_LDS_IDX_ACTIVE"):
                rec["lds_bank_conflict_frac"] = round(p1.get("SQ_LDS_BANK_CONFLICT", 0) / p1["SQ_LDS_IDX_ACTIVE"], 4)
            if p2.get("FETCH_SIZE") and ms:
                # FETCH_SIZE is in KiB; the PMC run's kernels take about the kernel-trace run's time
                rec["hbm_fetch_GB"] = round(p2["FETCH_SIZE"] * 1024 / 1e9, 3)
                rec["hbm_fetch_TBps"] = round(p2["FETCH_SIZE"] * 1024 / (ms / 1e3) / 1e12, 3)
            if p2.get("GRBM_GUI_ACTIVE") and p2.get("SQ_WAVES"):
                cyc = p2["GRBM_GUI_ACTIVE"] / 8.0
                rec["avg_waves_per_cu_cycle"] = round(p1.get("SQ_WAVE_CYCLES", 0) / max(1.0, cyc * 256) * 4, 3)
            rec["pmc_dispatches"] = [d1, d2]
            res["%s/%s" % (w, g)] = rec
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
