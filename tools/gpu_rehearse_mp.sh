#!/bin/bash
# The bench's N-rank path rehearsed on one GPU: torch.distributed.run with
# gloo (KGE_BENCH_BACKEND), ranks sharing the device. Checks the launch,
# barriers, max-over-ranks timing and the JSON line; the timings are not xGMI's.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp KGE_BENCH_BACKEND=gloo
OUT=gpurun_out/${1:-r04mp}
mkdir -p "$OUT"
port=29531
for cfg in "2 c2 auto" "4 c2 auto" "2 c2 owner" "2 c2 sparse"; do
  set -- $cfg
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $1 --workload $2 --exchange $3 --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_n$1_$2_$3.json" 2> "$OUT/bench_n$1_$2_$3.err" || { echo "N=$1 $2 $3 failed"; tail -30 "$OUT/bench_n$1_$2_$3.err"; exit 3; }
  head -c 400 "$OUT/bench_n$1_$2_$3.json"; echo
done
echo MP_OK
