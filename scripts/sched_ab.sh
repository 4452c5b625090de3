# A/B of scheduler-strategy variants of the N = 10 solve unit (scripts/variant_lib.sh NAME
# -mllvm -amdgpu-sched-strategy=S) against the default build: default-path parity, then the column
# kernel's event-timed duration vs batch, interleaved over 2 rounds.  usage: bash scripts/sched_ab.sh NAME ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp KERNELS=column
L=mav_trajectory_generation_cmake_amd/lib_var
for n in "$@"; do
  MTG_LIBRARY=$L/$n/libmav_trajectory_generation.so timeout -k 10 300 \
    python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "default or full_size or interior_waypoint or deterministic" --timeout 120 --timeout-method thread > gpurun_out/sched_$n.log 2>&1 \
    || { echo "parity FAILED for $n"; tail -20 gpurun_out/sched_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/sched_$n.log)"
done
for round in 1 2; do
  timeout -k 10 120 python scripts/sweep_kernels.py ${BATCHES:-1024 10000 131072} || exit $?
  for n in "$@"; do
    MTG_LIBRARY=$L/$n/libmav_trajectory_generation.so timeout -k 10 120 python scripts/sweep_kernels.py ${BATCHES:-1024 10000 131072} || exit $?
  done
done
