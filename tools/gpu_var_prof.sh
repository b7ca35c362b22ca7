#!/bin/bash
# rocprofv3 kernel stats of one bench leg per library variant (tools/variants.py).
# usage: gpu_var_prof.sh tag leg var [var ...]   ("main" = the in-tree library)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
LEG=$2
shift 2
mkdir -p "$OUT"
for v in "$@"; do
  LIBV=knowledge-graph-embedding_amd/KGE/_lib/libkge_var_$v.so
  [ "$v" = main ] && LIBV=knowledge-graph-embedding_amd/KGE/_lib/libkge_hip.so
  KGE_LIB=$PWD/$LIBV timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${LEG}_$v" -o run --output-format csv -- \
    python3 bench.py --workload $LEG --steps 50 --warmup 5 --no-cpu-baseline --no-hbm-point > "$OUT/bench_${LEG}_$v.json" 2> "$OUT/prof_${LEG}_$v.err" || { echo "rocprof $v failed"; tail -20 "$OUT/prof_${LEG}_$v.err"; exit 4; }
  echo "== $v"; python3 -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$OUT/bench_${LEG}_$v.json"
  find "$OUT/prof_${LEG}_$v" -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \; | head -7
done
echo VAR_OK
