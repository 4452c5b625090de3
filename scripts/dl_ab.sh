# DL kernel: GPU parity, then kernel time vs batch against the column kernel, then the variant
# libraries (scripts/variant_lib.sh) and trajectories-per-wave settings.  usage: bash scripts/dl_ab.sh [VARIANT ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "dl_kernel or golden_truth or bench_generator" \
  --timeout 120 --timeout-method thread > gpurun_out/dl_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/dl_tests.log
[ $rc -le 1 ] || exit $rc
KERNELS=column,dl timeout -k 10 200 python scripts/sweep_kernels.py ${BATCHES:-1024 4096 10000 32768 125000} || exit $?
for n in "$@"; do
  MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/$n/libmav_trajectory_generation.so KERNELS=dl timeout -k 10 120 \
    python scripts/sweep_kernels.py ${BATCHES:-1024 4096 10000 32768 125000} || exit $?
done
for t in ${TPWS:-}; do
  echo "MTG_DL_TPW=$t"
  MTG_DL_TPW=$t KERNELS=dl timeout -k 10 120 python scripts/sweep_kernels.py ${BATCHES:-1024 4096 10000 32768 125000} || exit $?
done
