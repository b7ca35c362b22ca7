#!/bin/bash
# TransR kernels A/B: tests matching -k EXPR, then the C4-TransR leg with the
# two-per-CU kernel (default) and the one-per-CU kernel (KGE_TRANSR_V1), each
# timed plainly and under rocprofv3 --kernel-trace --stats.
# usage: gpu_transr_ab.sh tag "pytest -k expr"
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread \
    -k "$2" > "$OUT/pytest_sel.log" 2>&1
  rc=$?; echo "selected tests: exit $rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_sel.log" | tail -20
  [ $rc -eq 0 ] || exit $rc
fi
for v in v2 v1; do
  if [ $v = v1 ]; then export KGE_TRANSR_V1=1; fi
  timeout -k 10 300 python3 bench.py --workload c4-transr --no-cpu-baseline --no-hbm-point > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" \
    || { echo "bench $v failed"; tail -20 "$OUT/bench_$v.err"; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r.get('kernel'), r.get('achieved'), r.get('frac'))" "$OUT/bench_$v.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o run --output-format csv -- \
    python3 bench.py --workload c4-transr --steps 30 --warmup 5 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/prof_$v.err" \
    || { echo "rocprof $v failed"; tail -20 "$OUT/prof_$v.err"; exit 4; }
  python3 tools/kstats.py "$OUT/prof_$v/run_kernel_stats.csv" 2>/dev/null | head -8
done
echo AB_OK
