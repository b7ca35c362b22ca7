#!/bin/bash
# One gpurun call: GPU parity tests, the bench line, a rocprofv3 kernel-trace
# summary and the two PMC passes (FETCH_SIZE / WRITE_SIZE) of the bench.
# usage: gpurun -- bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
echo "pytest_gpu exit $?" | tee -a "$OUT/status.txt"
tail -5 "$OUT/pytest_gpu.log"
grep -q -E "(Fatal|core dumped|Aborted|Segmentation)" "$OUT/pytest_gpu.log" && exit 3
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 4; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof failed"; tail -20 "$OUT/prof.err"; exit 5; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> "$OUT/pmc_fetch.err" || { echo "pmc fetch failed"; tail -20 "$OUT/pmc_fetch.err"; exit 6; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> "$OUT/pmc_write.err" || { echo "pmc write failed"; tail -20 "$OUT/pmc_write.err"; exit 7; }
find "$OUT" -name "*.csv" | head -20
echo ALL_OK
