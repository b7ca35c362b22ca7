#!/bin/bash
# Round-6 counters: per leg, HBM traffic per launch from two rocprofv3 --pmc
# passes (FETCH_SIZE, WRITE_SIZE; tools/pmc_traffic.py applies the gfx950
# correction) -> pmc_traffic_<leg>.json; L2 hit rate; the C4 legs' MFMA busy
# and wait counters. One --pmc pass per group (MI355X_MICROARCH.md rocprofv3).
# usage: gpu_pmc_r06.sh tag leg [leg ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
run() {   # run <dir> <leg> <counters...>
  local d=$1 w=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$d" -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/$d.err" \
    || { echo "pmc $d failed"; tail -5 "$OUT/$d.err"; exit 3; }
}
for w in "$@"; do
  run "fetch_$w" $w FETCH_SIZE
  run "write_$w" $w WRITE_SIZE
  python3 tools/pmc_traffic.py "$OUT/fetch_$w/run_counter_collection.csv" "$OUT/write_$w/run_counter_collection.csv" \
    "$OUT/pmc_traffic_$w.json" > /dev/null || exit 4
  run "l2_$w" $w TCC_HIT_sum TCC_MISS_sum
  echo "traffic $w ok"
done
for w in "$@"; do
  case $w in c4-*)
    run "sq_$w" $w SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
    echo "sq $w ok";;
  esac
done
echo PMC_OK
