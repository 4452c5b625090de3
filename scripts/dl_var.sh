# DL kernel variants (scripts/variant_lib.sh): parity of the first, then kernel time vs batch of each.
# usage: bash scripts/dl_var.sh VARIANT ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/$1/libmav_trajectory_generation.so timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "dl" --timeout 120 --timeout-method thread > gpurun_out/dl_var_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/dl_var_tests.log
[ $rc -le 1 ] || exit $rc
for n in "$@"; do
  MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/$n/libmav_trajectory_generation.so KERNELS=${KERNELS:-dl} timeout -k 10 120 \
    python scripts/sweep_kernels.py ${BATCHES:-1024 4096 10000 32768 125000} || exit $?
done
for t in ${TPWS:-}; do
  echo "MTG_DL_TPW=$t"
  MTG_DL_TPW=$t MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/$1/libmav_trajectory_generation.so KERNELS=dl \
    timeout -k 10 120 python scripts/sweep_kernels.py ${BATCHES:-1024 4096 10000 32768 125000} || exit $?
done
