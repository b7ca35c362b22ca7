#!/bin/bash
# Bench legs without profiling (one JSON line each). usage: gpu_legs.sh tag leg [leg ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
for w in "$@"; do
  timeout -k 10 400 python -u bench.py --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { echo "bench $w failed"; tail -20 "$OUT/bench_$w.err"; exit 3; }
  cat "$OUT/bench_$w.json"
done
echo LEGS_OK
