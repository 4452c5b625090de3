set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=mav_trajectory_generation_cmake_amd/lib_var
MTG_LIBRARY=$L/jacnt/libmav_trajectory_generation.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "jacobian or cost_at or time_sweep" --timeout 120 --timeout-method thread > gpurun_out/jab_t.log 2>&1 || { tail -20 gpurun_out/jab_t.log; exit 1; }
tail -1 gpurun_out/jab_t.log
for r in 1 2; do for v in jacplain jacnt; do
  MTG_LIBRARY=$L/$v/libmav_trajectory_generation.so timeout -k 10 120 python bench.py --workload config5 --no-cpu-baseline --steps 300 --warmup 100 > gpurun_out/jab_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/jab_$v.json')); r=d['roofline']; print('$v', '%.4g'%d['value'], 'kern %.4f iso %.4f'%(r['kernel_ms'], r['kernel_ms_isolated']))"
done; done
