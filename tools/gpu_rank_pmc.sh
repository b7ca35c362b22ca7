#!/bin/bash
# SQ counters of the ranking count pass (eval leg): rank_tile_kernel h / t side.
# usage: gpu_rank_pmc.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 300 python3 bench.py --workload eval --no-cpu-baseline > "$OUT/bench_eval.json" 2> "$OUT/bench_eval.err" \
  || { echo "eval failed"; tail -5 "$OUT/bench_eval.err"; exit 3; }
cat "$OUT/bench_eval.json"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 bench.py --workload eval --no-cpu-baseline > /dev/null 2> "$OUT/trace.err" \
  || { echo "trace failed"; tail -5 "$OUT/trace.err"; exit 3; }
cp "$OUT"/trace/run_kernel_stats.csv "$OUT/eval_kernel_stats.csv" 2>/dev/null || find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/eval_kernel_stats.csv" \;
cut -c1-140 "$OUT/eval_kernel_stats.csv" | head -8
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  -d "$OUT/pmc" -o run --output-format csv -- \
  python3 bench.py --workload eval --no-cpu-baseline > /dev/null 2> "$OUT/pmc.err" \
  || { echo "pmc failed"; tail -5 "$OUT/pmc.err"; exit 3; }
python3 - "$OUT" <<'PY' | tee "$OUT/rank_sq.txt"
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rank_" in r["Kernel_Name"]:
            acc[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    for c, v in sorted(cs.items()):
        print("%-48s %-24s n=%-3d %16.1f" % (k, c, len(v), max(v)))
PY
echo PMC_OK
