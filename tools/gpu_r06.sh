#!/bin/bash
# Round 6 iteration: pipelined-kernel diagnostic, GPU tests, default bench
# line, score-kernel variants on c2 / c2-50m. usage: gpu_r06.sh tag [variant ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/diag_pipe.py > "$OUT/diag.txt" 2>&1 || { echo "diag failed"; tail -20 "$OUT/diag.txt"; exit 1; }
cat "$OUT/diag.txt"
bash tools/gpu_round.sh "$TAG" "$@"
