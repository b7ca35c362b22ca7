#!/bin/bash
# Round evidence: bench lines (no profiler) of the given legs, each followed by
# a rocprofv3 kernel-trace/stats pass of the same leg. usage: gpu_evidence.sh tag "leg args" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for a in "$@"; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python3 bench.py --workload $a --no-cpu-baseline --no-hbm-point > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" \
    || { echo "bench $a failed"; tail -20 "$OUT/bench_$tag.err"; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d.get('value'))" "$OUT/bench_$tag.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$tag" -o run --output-format csv -- \
    python3 bench.py --workload $a --steps 30 --warmup 5 --no-cpu-baseline --no-hbm-point > /dev/null 2> "$OUT/prof_$tag.err" \
    || { echo "rocprof $a failed"; tail -20 "$OUT/prof_$tag.err"; exit 4; }
done
echo EVIDENCE_OK
