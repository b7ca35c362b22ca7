#!/bin/bash
# RESCAL: the GPU tests that reach it, the C4-RESCAL leg (x2), kernel stats
# and the score kernel's FETCH. usage: gpu_rescal_quick.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 500 python3 -u -m pytest tests/ -x -q -m gpu -k "rescal or RESCAL or Rescal" \
  --timeout 120 --timeout-method thread > "$OUT/pytest_rescal.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_rescal.log"; exit 3; }
tail -1 "$OUT/pytest_rescal.log"
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --workload c4-rescal --no-cpu-baseline > "$OUT/bench_c4-rescal_$rep.json" 2> "$OUT/err.txt" \
    || { echo "bench failed"; tail -5 "$OUT/err.txt"; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4-rescal', d['ms_per_step'])" "$OUT/bench_c4-rescal_$rep.json"
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 bench.py --workload c4-rescal --steps 50 --warmup 10 --no-cpu-baseline > /dev/null 2> "$OUT/trace.err" \
  || { echo "trace failed"; tail -5 "$OUT/trace.err"; exit 3; }
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/c4-rescal_kernel_stats.csv" \;
cut -c1-120 "$OUT/c4-rescal_kernel_stats.csv" | head -8
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc" -o run --output-format csv -- \
  python3 bench.py --workload c4-rescal --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/pmc.err" \
  || { echo "pmc failed"; tail -5 "$OUT/pmc.err"; exit 3; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if "kge" in k:
        print("%-60s FETCH_SIZE %.1f KiB/launch -> %.1f MB (x2 correction)" % (k, sum(v) / len(v), 2 * 1024 * sum(v) / len(v) / 1e6))
PY
echo RESCAL_OK
