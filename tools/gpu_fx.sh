#!/bin/bash
# The multi-GPU step rehearsed on one GPU (--force-exchange, and --loopback:
# every id through the exchange blocks), bench line + rocprofv3 kernel stats
# per leg. usage: gpu_fx.sh tag [legs...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
LEGS=${@:-c2 c5}
mkdir -p "$OUT"
for w in $LEGS; do
  for v in fx lb; do
    X="--force-exchange"
    [ $v = lb ] && X="--force-exchange --loopback"
    timeout -k 10 300 python -u bench.py --workload $w $X --no-cpu-baseline > "$OUT/bench_${w}_$v.json" 2> "$OUT/bench_${w}_$v.err" || { echo "bench $w $v failed"; tail -20 "$OUT/bench_${w}_$v.err"; exit 3; }
    cat "$OUT/bench_${w}_$v.json"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${w}_$v" -o run --output-format csv -- \
      python3 bench.py --workload $w $X --steps 50 --warmup 5 --no-cpu-baseline > /dev/null 2> "$OUT/prof_${w}_$v.err" || { echo "rocprof $w $v failed"; tail -20 "$OUT/prof_${w}_$v.err"; exit 4; }
    find "$OUT/prof_${w}_$v" -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-4 | head -16
  done
done
echo FX_OK
