#!/bin/bash
# C3 / C4 iteration: relation-family GPU tests, c4 legs with kernel stats,
# score-kernel variants on c3. usage: gpu_c34.sh tag [variant ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_tests.sh "$TAG" "RESCAL or Rescal or rescal or TransR or transr or rel" || exit 2
bash tools/gpu_bench_all.sh "$TAG" c4-rescal c4-transr || exit 3
if [ $# -gt 0 ]; then
  cp knowledge-graph-embedding_amd/KGE/_lib/libkge_hip.so knowledge-graph-embedding_amd/KGE/_lib/libkge_var_main.so
  timeout -k 10 500 python -u tools/variants.py run main "$@" -- --workload c3 > "$OUT/variants_c3.txt" 2>&1 || { echo "variants c3 failed"; cat "$OUT/variants_c3.txt"; exit 4; }
  cat "$OUT/variants_c3.txt"
fi
echo C34_OK
