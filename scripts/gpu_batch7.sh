set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pipelin or multi or host_arrays" > gpurun_out/pipe_tests.log 2>&1 || exit $?
timeout -k 10 400 python scripts/e2e_diag.py > gpurun_out/e2e_new.json 2> gpurun_out/e2e_new.err || exit $?
MTG_LIBRARY=$PWD/mav_trajectory_generation_cmake_amd/lib_var/pipe_old/libmav_trajectory_generation.so timeout -k 10 400 python scripts/e2e_diag.py > gpurun_out/e2e_old.json 2> gpurun_out/e2e_old.err || exit $?
