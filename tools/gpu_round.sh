#!/bin/bash
# One call: GPU parity tests, default bench line, then score-kernel variants
# (tools/variants.py) on c2 and c2-50m. usage: gpu_round.sh tag [variant ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_tests.sh "$TAG" || exit 2
timeout -k 10 300 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -20 "$OUT/bench_default.err"; exit 3; }
cat "$OUT/bench_default.json"
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u tools/variants.py run "$@" > "$OUT/variants_c2.txt" 2>&1 || { echo "variants c2 failed"; cat "$OUT/variants_c2.txt"; exit 4; }
  cat "$OUT/variants_c2.txt"
  timeout -k 10 400 python -u tools/variants.py run "$@" -- --workload c2-50m > "$OUT/variants_c2-50m.txt" 2>&1 || { echo "variants c2-50m failed"; cat "$OUT/variants_c2-50m.txt"; exit 5; }
  cat "$OUT/variants_c2-50m.txt"
fi
echo ROUND_OK
