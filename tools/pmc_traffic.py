"""Per-launch HBM traffic of the bench kernels from two rocprofv3 --pmc passes.

usage: python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (memory-side TCC_EA0 request
counters, Infinity-Cache hits included). gfx950 correction per
/opt/skills/guides/MI355X_MICROARCH.md (section HBM): FETCH_SIZE reports
exactly half the bytes of wide (16 B/lane) coalesced reads, which is the only
read shape these kernels issue (global_load_dwordx4 rows), so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""

import csv
import json
import sys
from collections import defaultdict

KERNELS = ("score_kernel", "update_kernel", "constrain_rows_kernel", "apply_kernel", "rel_item_kernel", "rel_dr_kernel",
           "rescal_apply_kernel", "transr2_kernel", "transr_kernel", "transr_proj_apply", "rescal_norms_kernel",
           "owner_merge_kernel", "owner_coef_kernel", "merge_chunk_kernel")


def short(name):
    # the kernel's own name (kge::<name><...>(...)), else the first listed
    # substring -- the longest first, so rescal_apply_kernel is not apply_kernel
    if "kge::" in name:
        base = name.split("kge::", 1)[1].split("(", 1)[0].split("<", 1)[0]
        if base.startswith("(anonymous namespace)::"):
            base = base.split("::", 1)[1]
        return base
    for k in sorted(KERNELS, key=len, reverse=True):
        if k in name:
            return k
    return None


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            k = short(row["Kernel_Name"])
            if k:
                acc[k].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    fetch, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
    write, nw = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {"unit": "bytes per launch", "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE "
           "counts half of 16 B/lane coalesced reads; MI355X_MICROARCH.md HBM)", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        out["kernels"][k] = {"fetch_size_kib": round(f, 1), "write_size_kib": round(w, 1),
                             "launches": [nf.get(k, 0), nw.get(k, 0)],
                             "hbm_bytes_per_launch": int((2 * f + w) * 1024)}
    s = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as fo:
            fo.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
