#!/bin/bash
# Round 4: the train() fast path (bound step, deferred epoch reads) -- its GPU
# tests, then the c1-train / c2-train legs.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "train or integration or rank" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc"
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in c2-train c1-train; do
  timeout -k 10 300 python3 bench.py --workload $w --epochs 2 > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { echo "$w failed"; tail -20 "$OUT/bench_$w.err"; exit 4; }
  cat "$OUT/bench_$w.json"
done
exit $rc
