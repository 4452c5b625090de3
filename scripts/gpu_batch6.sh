set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python bench.py --workload config4 --no-cpu-baseline > gpurun_out/bench_c4.json 2>gpurun_out/bench_c4.err || exit $?
bash scripts/r03_profiles.sh > gpurun_out/r03_profiles.log 2>&1
