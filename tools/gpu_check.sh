#!/bin/bash
# One GPU call: the GPU suite (optionally -k EXPR first), smoke, the default bench
# line, then extra bench legs. usage: gpu_check.sh tag [-k EXPR] [leg ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "$1" = "-k" ]; then
  timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread \
    -k "$2" > "$OUT/pytest_sel.log" 2>&1
  rc=$?; echo "selected tests: exit $rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest_sel.log" | tail -40
  [ $rc -eq 0 ] || exit $rc
  shift 2
fi
timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "gpu suite: exit $rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail "$OUT/smoke.log"; exit 5; }
cat "$OUT/smoke.log"
timeout -k 10 300 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -20 "$OUT/bench_default.err"; exit 6; }
head -c 600 "$OUT/bench_default.json"; echo
for a in "$@"; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python3 bench.py --workload $a --no-cpu-baseline --no-hbm-point > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" \
    || { echo "bench $a failed"; tail -20 "$OUT/bench_$tag.err"; exit 7; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r.get('kernel'), r.get('achieved'), r.get('frac'), r.get('frac_measured'))" "$OUT/bench_$tag.json"
done
echo CHECK_OK
