#!/bin/bash
# TransR iteration on the GPU box: the TransR parity tests, the phase profile
# (profiling build), the c4-transr bench line and its rocprof kernel stats.
# usage: gpurun -- bash tools/gpu_transr.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "transr or TransR" -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$OUT/pytest_transr.log" 2>&1
rc=$?
echo "pytest exit $rc"; tail -5 "$OUT/pytest_transr.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/transr_prof.py run > "$OUT/transr_phases.txt" 2>&1 || { tail -20 "$OUT/transr_phases.txt"; exit 5; }
cat "$OUT/transr_phases.txt"
timeout -k 10 300 python -u bench.py --workload c4-transr --no-cpu-baseline > "$OUT/bench_c4-transr.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 6; }
cat "$OUT/bench_c4-transr.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --workload c4-transr --steps 50 --warmup 5 --no-cpu-baseline > /dev/null 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 7; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec head -6 {} \;
echo TRANSR_OK
