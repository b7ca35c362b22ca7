#!/bin/bash
# r03d: full GPU tests, c4-rescal leg + rocprof, guard A/B on c2-50m
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r03d
mkdir -p $OUT
bash tools/gpu_tests.sh r03d || exit 2
timeout -k 10 300 python -u bench.py --workload c4-rescal --no-cpu-baseline > $OUT/bench_c4-rescal.json 2> $OUT/bench_c4-rescal.err || { tail -20 $OUT/bench_c4-rescal.err; exit 3; }
cat $OUT/bench_c4-rescal.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4r -o run --output-format csv -- python3 bench.py --workload c4-rescal --steps 50 --warmup 5 --no-cpu-baseline > /dev/null 2> $OUT/prof_c4r.err || { tail -20 $OUT/prof_c4r.err; exit 4; }
find $OUT/prof_c4r -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -14
timeout -k 10 300 python -u tools/variants.py run g2 g2off g2 g2off -- --workload c2-50m > $OUT/var50m.txt 2>&1; cat $OUT/var50m.txt
