#!/bin/bash
# One iteration on the GPU box: every GPU parity test, the TransR phase
# profile, then per leg a bench line (no CPU leg) and its rocprofv3 kernel
# stats. usage: gpurun -- bash tools/gpu_iter.sh tag leg [leg ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
[ -n "$NO_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc"; tail -4 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/transr_prof.py run > "$OUT/transr_phases.txt" 2>&1 || { tail -20 "$OUT/transr_phases.txt"; exit 5; }
grep -v amdgpu.ids "$OUT/transr_phases.txt"
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
    || { echo "bench $w failed"; tail -20 "$OUT/bench_$w.err"; exit 6; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], 'ms/step', d['value'])" "$OUT/bench_$w.json" $w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/prof_$w.err" \
    || { echo "rocprof $w failed"; tail -20 "$OUT/prof_$w.err"; exit 7; }
  find "$OUT/prof_$w" -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \; | head -8
done
echo ITER_OK
