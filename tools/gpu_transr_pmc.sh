#!/bin/bash
# SQ instruction / wait counters of the C4-TransR leg, two-per-CU kernel (v2)
# and the one-per-CU kernel (v1). usage: gpu_transr_pmc.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1
grep -o -E "SQ_[A-Z_0-9]*(MFMA|VALU|LDS)[A-Z_0-9]*" "$OUT/avail.txt" | sort -u | tr '\n' ' '; echo
for v in v2 v1; do
  if [ $v = v1 ]; then export KGE_TRANSR_V1=1; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    -d "$OUT/pmc_$v" -o run --output-format csv -- \
    python3 bench.py --workload c4-transr --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/pmc_$v.err" \
    || { echo "pmc $v failed"; tail -5 "$OUT/pmc_$v.err"; exit 3; }
  python3 - "$OUT/pmc_$v/run_counter_collection.csv" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if "transr" in r["Kernel_Name"] and "apply" not in r["Kernel_Name"]:
        acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    for c, v in sorted(cs.items()):
        print("%-40s %-28s %16.1f" % (k, c, sum(v) / len(v)))
PY
done
echo PMC_OK
