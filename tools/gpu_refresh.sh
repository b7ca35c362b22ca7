#!/bin/bash
# Round-end evidence refresh: every bench leg + rocprof kernel stats
# (gpu_bench_all.sh), then FETCH_SIZE / WRITE_SIZE passes for c2 and c2-50m
# turned into profiles-ready pmc_traffic JSON. usage: gpu_refresh.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_bench_all.sh "$TAG" || exit 2
for w in c2 c2-50m; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/pmc_${w}_$c" -o run --output-format csv -- \
      python3 bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/pmc_${w}_$c.err" \
      || { echo "pmc $w $c failed"; tail -5 "$OUT/pmc_${w}_$c.err"; exit 3; }
  done
  f=$(find "$OUT/pmc_${w}_FETCH_SIZE" -name "*counter_collection.csv" | head -n 1)
  g=$(find "$OUT/pmc_${w}_WRITE_SIZE" -name "*counter_collection.csv" | head -n 1)
  python3 tools/pmc_traffic.py "$f" "$g" "$OUT/pmc_traffic_$w.json" || exit 4
  cat "$OUT/pmc_traffic_$w.json"
done
echo REFRESH_OK
