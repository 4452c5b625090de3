set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ip_diag.py > gpurun_out/ipdiag_main.json 2>gpurun_out/ipdiag_main.err || exit $?
MTG_LIBRARY=$PWD/mav_trajectory_generation_cmake_amd/lib_var/ipnofb/libmav_trajectory_generation.so timeout -k 10 300 python scripts/ip_diag.py > gpurun_out/ipdiag_nofb.json 2>gpurun_out/ipdiag_nofb.err || exit $?
