"""Summarises rocprofv3 --pmc CSVs for one kernel: per-dispatch averages of every counter.

    python tools/pmc_summary.py gpurun_out/prof [kernel-substring]

Applies the gfx950 correction of MI355X_MICROARCH.md "HBM": FETCH_SIZE reports half
the bytes of a wide coalesced streaming read, so hbm_read_bytes = 2 * FETCH_SIZE KiB.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(root, kernel="scan_kernel"):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "pmc_*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    root = sys.argv[1]
    kernel = sys.argv[2] if len(sys.argv) > 2 else "scan_kernel"
    avg, n = summarise(root, kernel)
    for k in sorted(avg):
        print("%-28s %18.1f  (%d dispatches)" % (k, avg[k], n[k]))
    d = {}
    if "FETCH_SIZE" in avg:
        d["hbm_read_bytes"] = 2 * avg["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in avg:
        d["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "SQ_WAVE_CYCLES" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        d["valu_active_frac_of_wave_cycles"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
        d["wait_any_frac"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
        d["wait_inst_any_frac"] = avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
        d["active_inst_any_frac"] = avg["SQ_ACTIVE_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
