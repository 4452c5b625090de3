set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/debug_8030.py > gpurun_out/ab_default.log 2>&1 || exit $?
MTG_LIBRARY=$GRAFT_REPO_ROOT/mav_trajectory_generation_cmake_amd/lib_ieee/libmav_trajectory_generation.so timeout -k 10 200 python scripts/debug_8030.py > gpurun_out/ab_ieee.log 2>&1 || exit $?
