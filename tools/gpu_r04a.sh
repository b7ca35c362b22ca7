#!/bin/bash
# Round 4, first call: the GPU suite (incl. the new C4 full-size tests), the
# box's CPU share, and a kernel trace of the c2-train leg with its gaps.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p "$OUT"
{ echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; } > "$OUT/host.txt"
cat "$OUT/host.txt"
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc"
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2-train" -o run --output-format csv -- \
  python3 bench.py --workload c2-train --epochs 2 > "$OUT/bench_c2-train.json" 2> "$OUT/prof_c2-train.err" \
  || { echo "rocprof c2-train failed"; tail -20 "$OUT/prof_c2-train.err"; exit 4; }
cat "$OUT/bench_c2-train.json"
f=$(find "$OUT/prof_c2-train" -name "*kernel_trace.csv" | head -1)
python3 tools/kgaps.py "$f" > "$OUT/c2-train_gaps.txt"; cat "$OUT/c2-train_gaps.txt"
exit $rc
