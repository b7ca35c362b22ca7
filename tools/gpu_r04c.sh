#!/bin/bash
# Round 4: owner-side scoring -- its GPU tests (world 1 RCCL, two ranks on one
# GPU), then C5 rehearsals at N=1 (owner, sparse) and C2 (dense, owner, sparse).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "owner or world1 or two_ranks or overflow" -x > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc"
grep -E "FAILED|ERROR|passed|failed|Error" "$OUT/pytest_gpu.log" | tail -30
[ $rc -eq 0 ] || exit $rc
for a in "c5 --force-exchange --exchange owner" "c5 --force-exchange --exchange owner --loopback" \
         "c5 --force-exchange --exchange sparse" "c2 --force-exchange --exchange owner" \
         "c2 --force-exchange --exchange sparse" "c2 --force-exchange --exchange dense"; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python3 bench.py --workload $a --steps 50 --warmup 5 --no-cpu-baseline --no-hbm-point \
    > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { echo "$a failed"; tail -20 "$OUT/bench_$tag.err"; exit 4; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['config'].get('exchange'), {k: v.get('ms') for k, v in d['roofline']['kernels'].items()})" "$OUT/bench_$tag.json"
done
