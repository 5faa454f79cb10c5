"""Sum rocprofv3 --pmc counter CSVs over the dispatches of one kernel (name substring) and derive
utilisation ratios. python tools/pmc_summary.py <kernel-substring> <pmc-dir>"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    pat, root = sys.argv[1], sys.argv[2]
    tot = defaultdict(float)
    disp = set()
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if pat not in r.get("Kernel_Name", ""):
                continue
            disp.add((f, r.get("Dispatch_Id")))
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    out = dict(sorted(tot.items()))
    out["dispatches"] = len(disp)
    if tot.get("GRBM_GUI_ACTIVE"):
        cyc = tot["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
        if tot.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            out["mfma_busy_per_simd"] = round(tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc), 4)
    if tot.get("TCC_HIT_sum") is not None and tot.get("TCC_MISS_sum") is not None:
        out["l2_hit_rate"] = round(tot["TCC_HIT_sum"] / max(1.0, tot["TCC_HIT_sum"] + tot["TCC_MISS_sum"]), 4)
    if tot.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac"] = round(tot.get("SQ_LDS_BANK_CONFLICT", 0.0) / tot["SQ_LDS_IDX_ACTIVE"], 4)
    if tot.get("SQ_WAVES"):
        for key in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if key in tot:
                out[key.lower()[3:] + "_per_wave"] = round(tot[key] / tot["SQ_WAVES"], 1)
    if tot.get("SQ_WAVE_CYCLES"):
        out["wait_inst_lds_frac"] = round(tot.get("SQ_WAIT_INST_LDS", 0.0) / tot["SQ_WAVE_CYCLES"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
