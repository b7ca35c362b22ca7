#!/bin/bash
# rank + stream tests, then the eval leg with its kernel stats. usage: gpu_it9.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_rank.py tests/test_gpu_stream.py -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/$T/pytest_rank.log 2>&1 || { tail -40 gpurun_out/$T/pytest_rank.log; exit 2; }
tail -2 gpurun_out/$T/pytest_rank.log
timeout -k 10 300 python -u bench.py --workload eval > gpurun_out/$T/bench_eval.json 2> gpurun_out/$T/bench_eval.err \
  || { tail -20 gpurun_out/$T/bench_eval.err; exit 3; }
cat gpurun_out/$T/bench_eval.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof_eval -o run --output-format csv -- \
  python3 bench.py --workload eval --no-cpu-baseline > /dev/null 2> gpurun_out/$T/prof_eval.err || { tail -20 gpurun_out/$T/prof_eval.err; exit 4; }
find gpurun_out/$T/prof_eval -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
echo IT9_OK
