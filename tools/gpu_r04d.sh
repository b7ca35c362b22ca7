#!/bin/bash
# Round 4 (re-entry): full GPU suite + smoke, the default bench line under
# rocprof, then the multi-GPU rehearsals at N=1 (owner / sparse / dense).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04d
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc"
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail "$OUT/smoke.log"; exit 5; }
cat "$OUT/smoke.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run --output-format csv -- \
  python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -20 "$OUT/bench_default.err"; exit 4; }
cat "$OUT/bench_default.json"
for a in "c5 --force-exchange --exchange owner" "c5 --force-exchange --exchange owner --loopback" \
         "c5 --force-exchange --exchange sparse" "c2 --force-exchange --exchange owner" \
         "c2 --force-exchange --exchange sparse" "c2 --force-exchange --exchange dense"; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python3 bench.py --workload $a --steps 50 --warmup 5 --no-cpu-baseline --no-hbm-point \
    > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { echo "$a failed"; tail -20 "$OUT/bench_$tag.err"; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['config'].get('exchange'), {k: v.get('ms') for k, v in d['roofline']['kernels'].items()})" "$OUT/bench_$tag.json"
done
exit $rc
