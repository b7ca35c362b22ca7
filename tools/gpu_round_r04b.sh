#!/bin/bash
# Round-4 evidence, part 2: score/update variants on c2, the multi-GPU
# rehearsals, the train() and evaluate() legs.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/variants.py run base s32 u12 s128 > gpurun_out/variants_r04.txt 2>&1
cat gpurun_out/variants_r04.txt
bash tools/gpu_evidence.sh r04c "c5" "c5 --force-exchange --exchange owner" "c5 --force-exchange --exchange owner --loopback" \
  "c5 --force-exchange --exchange sparse" "c2 --force-exchange --exchange dense" "c2 --force-exchange --exchange owner" \
  "c2 --force-exchange --exchange sparse" || exit 3
for w in c1-train c2-train eval; do
  timeout -k 10 300 python3 bench.py --workload $w > "gpurun_out/r04c/bench_$w.json" 2> "gpurun_out/r04c/bench_$w.err" || { echo "$w failed"; tail -20 "gpurun_out/r04c/bench_$w.err"; exit 4; }
  head -c 600 "gpurun_out/r04c/bench_$w.json"; echo
done
echo PART2_OK
