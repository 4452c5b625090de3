set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ip_diag.py > gpurun_out/ipdiag_loop.json 2>gpurun_out/ipdiag_loop.err || exit $?
MTG_LIBRARY=$PWD/mav_trajectory_generation_cmake_amd/lib_var/ipw2/libmav_trajectory_generation.so timeout -k 10 300 python scripts/ip_diag.py > gpurun_out/ipdiag_w2.json 2>gpurun_out/ipdiag_w2.err || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ip" > gpurun_out/ip_tests.log 2>&1
