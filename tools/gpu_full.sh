#!/bin/bash
# Full GPU suite + smoke, then kernel traces of bench legs (quoted arg strings).
# usage: gpu_full.sh tag ["leg args" ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc"
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail "$OUT/smoke.log"; exit 5; }
cat "$OUT/smoke.log"
[ $# -gt 0 ] && bash tools/gpu_trace.sh "$TAG" "$@"
exit 0
