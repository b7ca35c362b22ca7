#!/bin/bash
# quick GPU iteration: parity tests, phase profile, bench (no CPU leg)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc"; tail -15 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/phase_prof.py run --score-wgs 512 --update-wgs 3686 > "$OUT/phase.txt" 2>&1 || { tail -20 "$OUT/phase.txt"; exit 5; }
cat "$OUT/phase.txt"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 6; }
cat "$OUT/bench.json"
if [ -f knowledge-graph-embedding_amd/KGE/_lib/libkge_hip_prof16.so ]; then
  KGE_PROF_LIB=libkge_hip_prof16.so timeout -k 10 200 python -u tools/phase_prof.py run --score-wgs 512 --update-wgs 3686 > "$OUT/phase16.txt" 2>&1 || { tail -20 "$OUT/phase16.txt"; exit 7; }
  echo "== variant (U=16)"; cat "$OUT/phase16.txt"
fi
