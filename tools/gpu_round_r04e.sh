#!/bin/bash
# Round-4 evidence, part 3 (after the device histograms and the batch ring):
# GPU suite + smoke, the default bench line under rocprof, the train() and
# evaluate() legs, the C5 owner rehearsals.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04e
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
for w in c1-train c2-train eval; do
  timeout -k 10 300 python3 bench.py --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { echo "$w failed"; tail -20 "$OUT/bench_$w.err"; exit 4; }
  head -c 900 "$OUT/bench_$w.json"; echo
done
bash tools/gpu_evidence.sh r04e "c5 --force-exchange --exchange owner" "c5 --force-exchange --exchange owner --loopback" || exit 3
echo R04E_OK
