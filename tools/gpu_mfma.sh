#!/bin/bash
# MFMA utilisation of the C4 legs: SQ_VALU_MFMA_BUSY_CYCLES against
# GRBM_GUI_ACTIVE (one --pmc pass per leg). usage: gpu_mfma.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || { echo "list failed"; tail -5 "$OUT/avail.txt"; exit 2; }
grep -i -E "mfma|SQ_BUSY_CU|GRBM_GUI_ACTIVE" "$OUT/avail.txt" | head -40
for w in c4-transr c4-rescal; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d "$OUT/mfma_$w" -o run --output-format csv -- \
    python3 bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> "$OUT/mfma_$w.err" \
    || { echo "pmc $w failed"; tail -5 "$OUT/mfma_$w.err"; exit 3; }
  echo "pass $w ok"
done
echo MFMA_OK
