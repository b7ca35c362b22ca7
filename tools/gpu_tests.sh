#!/bin/bash
# GPU parity tests only. usage: gpu_tests.sh tag [pytest -k expr]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > "$OUT/pytest_gpu.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
rc=$?
echo "pytest exit $rc"
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest_gpu.log" | tail -30
exit $rc
