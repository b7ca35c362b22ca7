#!/bin/bash
# GPU tests matching a -k expression, then kernel traces of bench legs.
# usage: gpu_quick.sh tag "pytest -k expr" ["leg args" ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "$K" > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  echo "pytest exit $rc"
  grep -E "FAILED|ERROR|passed|failed|Error" "$OUT/pytest_gpu.log" | tail -30
  [ $rc -eq 0 ] || exit $rc
fi
[ $# -gt 0 ] && bash tools/gpu_trace.sh "$TAG" "$@"
exit 0
