"""MFMA utilisation per kernel from a rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (tools/gpu_mfma.sh).

usage: python tools/mfma_util.py <counter_collection.csv> [filter] ...

GRBM_GUI_ACTIVE is reported summed over the 8 XCDs, so a dispatch's cycles are
GUI / 8; utilisation = MFMA busy cycles / (GUI / 8 * 1024 SIMDs), averaged over
the kernel's dispatches (rocprofv3's MfmaUtil expression).
"""
import csv
import json
import sys
from collections import defaultdict


def util(path, flt=("transr", "rel_")):
    per = defaultdict(lambda: defaultdict(dict))
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if not any(s in name for s in flt):
                continue
            per[name][r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    out = {}
    for name, ds in per.items():
        busy = [d["SQ_VALU_MFMA_BUSY_CYCLES"] for d in ds.values() if "SQ_VALU_MFMA_BUSY_CYCLES" in d]
        gui = [d["GRBM_GUI_ACTIVE"] for d in ds.values() if "GRBM_GUI_ACTIVE" in d]
        if not busy or not gui:
            continue
        b, g = sum(busy) / len(busy), sum(gui) / len(gui) / 8.0
        out[name.split("(")[0]] = {"mfma_busy_cycles": b, "kernel_cycles_per_xcd": round(g),
                                   "mfma_util_pct": round(100.0 * b / (g * 1024.0), 1), "dispatches": len(busy)}
    return out


if __name__ == "__main__":
    print(json.dumps({p: util(p) for p in sys.argv[1:]}, indent=1))
