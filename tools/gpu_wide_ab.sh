#!/bin/bash
# Wide score-kernel variants (tools/variants.py buildfull) against the shipped
# library on C3 and C5. usage: gpu_wide_ab.sh tag variant...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
  for leg in c3 c5; do
    timeout -k 10 200 python3 bench.py --workload $leg --no-cpu-baseline --no-hbm-point > "$OUT/base_${leg}_$rep.json" 2>/dev/null || exit 3
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline'].get('kernels') or {}; print('base', sys.argv[2], d['ms_per_step'], k)" "$OUT/base_${leg}_$rep.json" $leg
    timeout -k 10 600 python3 tools/variants.py run "$@" -- --workload $leg || exit 3
  done
done
