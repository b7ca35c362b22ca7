#!/bin/bash
# Ranking: GPU rank tests, the eval leg, its kernel stats. usage: gpu_rank.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rank.py -x -q -m gpu --timeout 120 --timeout-method thread \
  > "$OUT/pytest_rank.log" 2>&1 || { echo "rank tests failed"; tail -30 "$OUT/pytest_rank.log"; exit 3; }
tail -2 "$OUT/pytest_rank.log"
timeout -k 10 300 python3 bench.py --workload eval --no-cpu-baseline > "$OUT/bench_eval.json" 2> "$OUT/bench_eval.err" \
  || { echo "eval failed"; tail -5 "$OUT/bench_eval.err"; exit 3; }
cat "$OUT/bench_eval.json"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 bench.py --workload eval --no-cpu-baseline > /dev/null 2> "$OUT/trace.err" \
  || { echo "trace failed"; tail -5 "$OUT/trace.err"; exit 3; }
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/eval_kernel_stats.csv" \;
cut -c1-150 "$OUT/eval_kernel_stats.csv" | head -10
echo RANK_OK
