set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "magnitude" > gpurun_out/ext_tests.log 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_extrema.py > gpurun_out/bench_extrema.json 2>gpurun_out/bench_extrema.err || exit $?
MTG_LIBRARY=$PWD/mav_trajectory_generation_cmake_amd/lib_var/extL8/libmav_trajectory_generation.so timeout -k 10 200 python scripts/bench_extrema.py > gpurun_out/bench_extrema_L8.json 2>gpurun_out/bench_extrema_L8.err || exit $?
timeout -k 10 200 python scripts/bench_extrema.py > gpurun_out/bench_extrema_2.json 2>gpurun_out/bench_extrema.err || exit $?
