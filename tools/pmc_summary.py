"""Per-kernel mean of every PMC counter collected by tools/gpu_pmc.sh.

usage: python tools/pmc_summary.py <dir with pmc*/ subdirs>

Prints one line per (kernel, counter): mean value per dispatch. FETCH_SIZE is
also shown doubled (gfx950 reports half the bytes of 16 B/lane coalesced
reads, MI355X_MICROARCH.md HBM section) and the L2 hit rate is derived from
TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum).
"""

import csv
import glob
import os
import sys
from collections import defaultdict

KERNELS = ("score_kernel", "update_kernel", "constrain_rows_kernel", "apply_kernel", "rank_count_kernel")


def short(name):
    """kge kernels by their short name (templates folded); others dropped."""
    for k in KERNELS:
        if k in name:
            return k
    if "kge::" in name:
        base = name.split("kge::", 1)[1]
        for sep in ("<", "("):
            base = base.split(sep, 1)[0]
        return base
    return None


def main():
    root = sys.argv[1]
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row.get("Kernel_Name", ""))
                if k:
                    vals[(k, row["Counter_Name"])].append(float(row["Counter_Value"]))
    mean = {key: sum(v) / len(v) for key, v in vals.items()}
    for (k, c), m in sorted(mean.items()):
        extra = ""
        if c == "FETCH_SIZE":
            extra = "  (x2 = %.1f MB)" % (2 * m / 1024.0)
        elif c == "WRITE_SIZE":
            extra = "  (%.1f MB)" % (m / 1024.0)
        print("%-22s %-22s %16.1f%s" % (k, c, m, extra))
    for k in KERNELS:
        h, mi = mean.get((k, "TCC_HIT_sum")), mean.get((k, "TCC_MISS_sum"))
        if h is not None and mi is not None and h + mi > 0:
            print("%-22s L2 hit rate %.3f" % (k, h / (h + mi)))


if __name__ == "__main__":
    main()
