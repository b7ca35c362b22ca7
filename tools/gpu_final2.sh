#!/bin/bash
# every GPU test, smoke(), the default bench line and its rocprof kernel stats. usage: gpu_final2.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
T=$1
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 2; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 3; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 4; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_default" -o run --output-format csv -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > "$OUT/prof_default.json" 2> "$OUT/prof_default.err" \
  || { tail -20 "$OUT/prof_default.err"; exit 5; }
find "$OUT/prof_default" -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \; | head -4
echo FINAL2_OK
