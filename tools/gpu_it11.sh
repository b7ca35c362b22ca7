#!/bin/bash
# TransR + rank tests, TransR phases + c4-transr leg, eval leg. usage: gpu_it11.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "transr or TransR or rank" -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 2; }
tail -2 gpurun_out/$T/pytest.log
NO_TESTS=1 timeout -k 10 400 bash tools/gpu_iter.sh $T c4-transr || exit 3
timeout -k 10 300 bash tools/gpu_it9.sh ${T}e > /dev/null 2>&1; tail -3 gpurun_out/${T}e/pytest_rank.log; cat gpurun_out/${T}e/bench_eval.json
find gpurun_out/${T}e/prof_eval -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \; | head -5
echo IT11_OK
