#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 --pmc pass per counter
# group; MI355X_MICROARCH.md HBM/rocprofv3 section). usage: gpu_pmc.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- \
    python3 bench.py --workload ${2:-c2} --steps 10 --warmup 3 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/pmc$i.err" || { echo "pmc pass $i ($grp) failed"; tail -5 "$OUT/pmc$i.err"; exit 3; }
  echo "pass $i ok: $grp"
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.txt" && cat "$OUT/pmc_summary.txt"
