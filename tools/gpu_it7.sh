#!/bin/bash
# score-kernel phases at C2 and C2-50M, TransR phases + c4-transr leg,
# c2-train leg. usage: gpu_it7.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u tools/phase_prof.py run --score-wgs 512 --update-wgs 3686 > gpurun_out/$T/phase_c2.txt 2>&1 \
  || { tail -20 gpurun_out/$T/phase_c2.txt; exit 2; }
grep -v amdgpu.ids gpurun_out/$T/phase_c2.txt
timeout -k 10 300 python -u tools/phase_prof.py run --entities 50000000 --score-wgs 512 --update-wgs 16576 \
  > gpurun_out/$T/phase_c2-50m.txt 2>&1 || { tail -20 gpurun_out/$T/phase_c2-50m.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/$T/phase_c2-50m.txt
NO_TESTS=1 timeout -k 10 400 bash tools/gpu_iter.sh $T c4-transr || exit 4
timeout -k 10 300 python -u bench.py --workload c2-train > gpurun_out/$T/bench_c2-train.json 2> gpurun_out/$T/bench_c2-train.err \
  || { tail -20 gpurun_out/$T/bench_c2-train.err; exit 5; }
cat gpurun_out/$T/bench_c2-train.json

timeout -k 10 400 bash tools/gpu_pmc.sh ${T}p c2-50m || exit 6
for a in "--force-exchange" "--force-exchange --loopback"; do
  timeout -k 10 300 python -u bench.py --workload c5 $a --no-cpu-baseline > gpurun_out/$T/bench_c5.json 2> gpurun_out/$T/bench_c5.err \
    || { tail -20 gpurun_out/$T/bench_c5.err; exit 7; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', sys.argv[2], d['ms_per_step'], d['value'])" gpurun_out/$T/bench_c5.json "$a"
done
echo IT7_DONE
