#!/bin/bash
# every GPU test, then the train-entry legs (c1-train, c2-train) and the
# c2-train kernel trace. usage: gpu_it6.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/$T/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$T/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/$T/pytest_gpu.log
for w in c1-train c2-train; do
  timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/$T/bench_$w.json 2> gpurun_out/$T/bench_$w.err \
    || { tail -20 gpurun_out/$T/bench_$w.err; exit 3; }
  cat gpurun_out/$T/bench_$w.json
done
timeout -k 10 300 bash tools/gpu_trace_train.sh $T || exit 4
echo IT6_OK
