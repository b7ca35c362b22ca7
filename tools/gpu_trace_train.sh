#!/bin/bash
# Kernel trace of the c2-train leg (KGEModel.train): per-batch kernels and the
# gaps between them. usage: gpu_trace_train.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2-train" -o run --output-format csv -- \
  python3 bench.py --workload c2-train --epochs 1 > "$OUT/bench_c2-train.json" 2> "$OUT/prof_c2-train.err" \
  || { echo "rocprof c2-train failed"; tail -20 "$OUT/prof_c2-train.err"; exit 4; }
cat "$OUT/bench_c2-train.json"
find "$OUT/prof_c2-train" -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
echo TRACE_OK
