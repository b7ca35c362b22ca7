#!/bin/bash
# TransR: the GPU tests that reach transr2_kernel, the C4-TransR leg (x2) and
# the phase profile. usage: gpu_transr_quick.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_step.py -x -q -m gpu -k "transr or TransR" \
  --timeout 120 --timeout-method thread > "$OUT/pytest_transr.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_transr.log"; exit 3; }
tail -1 "$OUT/pytest_transr.log"
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --workload c4-transr --no-cpu-baseline > "$OUT/bench_c4-transr_$rep.json" 2> "$OUT/err.txt" \
    || { echo "bench failed"; tail -5 "$OUT/err.txt"; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4-transr', d['ms_per_step'])" "$OUT/bench_c4-transr_$rep.json"
done
timeout -k 10 300 python3 tools/transr_prof.py run > "$OUT/transr_phases_v2.txt" 2>&1 || { echo "prof failed"; tail -5 "$OUT/transr_phases_v2.txt"; exit 3; }
cat "$OUT/transr_phases_v2.txt"
echo TR_OK
