#!/bin/bash
# Bench line + rocprofv3 kernel stats per leg. usage: gpu_prof.sh tag leg [leg ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-hbm-point > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { echo "bench $w failed"; tail -20 "$OUT/bench_$w.err"; exit 3; }
  cat "$OUT/bench_$w.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/prof_$w.err" || { echo "rocprof $w failed"; tail -20 "$OUT/prof_$w.err"; exit 4; }
  find "$OUT/prof_$w" -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
done
echo PROF_OK
