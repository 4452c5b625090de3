# A/B of variant libraries (scripts/variant_lib.sh): GPU parity on the default-path tests, then
# the column kernel's time vs batch, interleaved over 2 rounds.  usage: bash scripts/var_ab.sh NAME ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp KERNELS=${KERNELS:-column}
for n in $( [ -z "$NOPARITY" ] && echo "$@" ); do
  MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/$n/libmav_trajectory_generation.so timeout -k 10 300 \
    python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "${PARITY_K:-default or full_size or paths_agree or interior_waypoint or deterministic or sharded or status}" --timeout 120 --timeout-method thread > gpurun_out/var_$n.log 2>&1 \
    || { echo "parity FAILED for $n"; tail -20 gpurun_out/var_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/var_$n.log)"
done
for round in 1 2; do
  for n in "$@"; do
    MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/$n/libmav_trajectory_generation.so timeout -k 10 120 \
      python scripts/sweep_kernels.py ${BATCHES:-1024 8192 10000} || exit $?
  done
done
