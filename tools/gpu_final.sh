#!/bin/bash
# Round-end evidence: every GPU test, smoke(), the default bench line, its
# rocprof kernel stats, then every leg + kernel stats and the c2 / c2-50m PMC
# traffic (gpu_refresh.sh). usage: gpu_final.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
T=$1
OUT=gpurun_out/$T
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 2; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 3; }
tail -2 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 4; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_default" -o run --output-format csv -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > "$OUT/prof_default.json" 2> "$OUT/prof_default.err" \
  || { tail -20 "$OUT/prof_default.err"; exit 5; }
timeout -k 10 1200 bash tools/gpu_refresh.sh "$T" || exit 6
for w in c1-train c2-train eval; do
  timeout -k 10 300 python -u bench.py --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 7; }
  cat "$OUT/bench_$w.json"
done
for a in "--force-exchange" "--force-exchange --loopback"; do
  n=$(echo "$a" | tr -d ' -')
  timeout -k 10 300 python -u bench.py --workload c5 $a --no-cpu-baseline > "$OUT/bench_c5_$n.json" 2> "$OUT/bench_c5_$n.err" || { tail -20 "$OUT/bench_c5_$n.err"; exit 8; }
  cat "$OUT/bench_c5_$n.json"
done
timeout -k 10 300 python -u bench.py --workload c2 --force-exchange --no-cpu-baseline > "$OUT/bench_c2_fx.json" 2> "$OUT/bench_c2_fx.err" || { tail -20 "$OUT/bench_c2_fx.err"; exit 9; }
cat "$OUT/bench_c2_fx.json"
timeout -k 10 200 python -u tools/transr_prof.py run > "$OUT/transr_phases.txt" 2>&1 || { tail -20 "$OUT/transr_phases.txt"; exit 10; }
grep -v amdgpu.ids "$OUT/transr_phases.txt"
echo FINAL_OK
