#!/bin/bash
# Kernel trace + per-kernel averages / gaps of bench legs given as quoted
# argument strings. usage: gpu_trace.sh tag "leg args" ["leg args" ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
for a in "$@"; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$tag" -o run --output-format csv -- \
    python3 bench.py --workload $a --steps 30 --warmup 5 --no-cpu-baseline --no-hbm-point \
    > "$OUT/bench_$tag.json" 2> "$OUT/prof_$tag.err" || { echo "rocprof $a failed"; tail -20 "$OUT/prof_$tag.err"; exit 4; }
  f=$(find "$OUT/prof_$tag" -name "*kernel_trace.csv" | head -1)
  python3 tools/kgaps.py "$f" > "$OUT/gaps_$tag.txt"
  echo "== $a"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'])" "$OUT/bench_$tag.json"
  head -25 "$OUT/gaps_$tag.txt"
done
echo TRACE_OK
