#!/bin/bash
# GPU tests matching -k EXPR, then per leg: a bench line, a kernel trace
# (rocprofv3 --kernel-trace --stats) and FETCH/WRITE PMC passes.
# usage: gpu_leg_prof.sh tag "pytest -k expr" leg [leg ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread \
    -k "$K" > "$OUT/pytest_sel.log" 2>&1
  rc=$?; echo "selected tests: exit $rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_sel.log" | tail -20
  [ $rc -eq 0 ] || exit $rc
fi
for w in "$@"; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --no-hbm-point > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { echo "bench $w failed"; tail -20 "$OUT/bench_$w.err"; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r.get('kernel'), r.get('achieved'), r.get('frac'), r.get('frac_measured'))" "$OUT/bench_$w.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 30 --warmup 5 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/prof_$w.err" \
    || { echo "rocprof $w failed"; tail -20 "$OUT/prof_$w.err"; exit 4; }
  python3 tools/kstats.py "$OUT/prof_$w/run_kernel_stats.csv" 2>/dev/null | head -14 || head -12 "$OUT/prof_$w/run_kernel_stats.csv"
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/pmc_$w$i" -o run --output-format csv -- \
      python3 bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/pmc_$w$i.err" \
      || { echo "pmc $w $grp failed"; tail -5 "$OUT/pmc_$w$i.err"; exit 5; }
  done
  python3 tools/pmc_traffic.py "$OUT/pmc_${w}1/run_counter_collection.csv" "$OUT/pmc_${w}2/run_counter_collection.csv" "$OUT/pmc_traffic_$w.json" > /dev/null && head -c 1500 "$OUT/pmc_traffic_$w.json"; echo
done
echo LEG_OK
