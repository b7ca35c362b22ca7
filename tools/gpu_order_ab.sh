#!/bin/bash
# A/B of the relation-ordered, XCD-grouped positives (RESCAL / TransR train
# steps) against batch order (KGE_NO_POS_ORDER). usage: gpu_order_ab.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_step.py -x -q -m gpu -k "rescal or transr or RESCAL or TransR" \
  --timeout 120 --timeout-method thread > "$OUT/pytest_sel.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/pytest_sel.log"; exit 3; }
tail -1 "$OUT/pytest_sel.log"
for rep in 1 2; do
  for leg in c4-rescal c4-transr; do
    for v in order batch; do
      if [ $v = batch ]; then export KGE_NO_POS_ORDER=1; else unset KGE_NO_POS_ORDER; fi
      timeout -k 10 200 python3 bench.py --workload $leg --no-cpu-baseline > "$OUT/bench_${leg}_${v}_$rep.json" 2> "$OUT/err_$leg.txt" \
        || { echo "bench $leg $v failed"; tail -5 "$OUT/err_$leg.txt"; exit 3; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'])" \
        "$OUT/bench_${leg}_${v}_$rep.json" $leg $v
    done
  done
done
unset KGE_NO_POS_ORDER
for leg in c4-rescal c4-transr; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$leg" -o run --output-format csv -- \
    python3 bench.py --workload $leg --steps 50 --warmup 10 --no-cpu-baseline > /dev/null 2> "$OUT/trace_$leg.err" \
    || { echo "trace failed"; tail -5 "$OUT/trace_$leg.err"; exit 3; }
  find "$OUT/trace_$leg" -name "*kernel_stats.csv" -exec cp {} "$OUT/${leg}_kernel_stats.csv" \;
  cut -c1-120 "$OUT/${leg}_kernel_stats.csv" | head -6
done
echo AB_OK
