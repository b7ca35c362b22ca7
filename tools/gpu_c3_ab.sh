cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06z
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --workload c3 --no-cpu-baseline --no-hbm-point > gpurun_out/r06z/base_$rep.json 2>/dev/null || exit 3
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline']['kernels']; print('base', d['ms_per_step'], k['score_kernel']['ms'], k['update_kernel']['ms'])" gpurun_out/r06z/base_$rep.json
  timeout -k 10 300 python3 tools/variants.py run u4 -- --workload c3 || exit 3
  timeout -k 10 300 python3 tools/variants.py run u4 -- --workload c2 || exit 3
done
