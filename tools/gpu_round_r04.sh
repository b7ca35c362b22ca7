#!/bin/bash
# Round-4 evidence, part 1: GPU suite + smoke, the default bench line under
# rocprof, then the single-GPU legs.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail "$OUT/smoke.log"; exit 5; }
cat "$OUT/smoke.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_default" -o run --output-format csv -- \
  python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -20 "$OUT/bench_default.err"; exit 6; }
cat "$OUT/bench_default.json"
bash tools/gpu_evidence.sh r04c c1 c3 c4-rescal c4-transr c2-50m
