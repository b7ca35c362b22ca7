#!/bin/bash
# TransR parity tests, TransR phases + c4-transr leg, score-kernel variants on
# c2-50m and c2, and the c2-train kernel trace. usage: gpu_it5.sh tag
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "transr or TransR" -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/$T/pytest_transr.log 2>&1 || { tail -30 gpurun_out/$T/pytest_transr.log; exit 2; }
tail -2 gpurun_out/$T/pytest_transr.log
NO_TESTS=1 timeout -k 10 400 bash tools/gpu_iter.sh $T c4-transr || exit 3
timeout -k 10 500 bash tools/gpu_var_prof.sh ${T}v c2-50m kr4 pf1 sr16 sr12 || exit 4
timeout -k 10 500 bash tools/gpu_var_prof.sh ${T}v c2 kr4 pf1 sr16 sr12 || exit 5
timeout -k 10 300 bash tools/gpu_trace_train.sh $T || exit 6
echo IT5_OK
