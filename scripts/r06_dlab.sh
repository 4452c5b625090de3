# Round 6: DL-kernel variant libraries -- the solve bench over vertex patterns (as r06ab.sh) and the
# DL-kernel parity tests on each variant.  usage: bash scripts/r06_dlab.sh VARIANT ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
EVID=${EVID:-r06dlab} PATTERNS="${PATTERNS:-generator accel-ends}" bash scripts/r06ab.sh "$@" || exit $?
for v in "$@"; do
  MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/$v/libmav_trajectory_generation.so timeout -k 10 600 \
    python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread \
    -k "dl_ or golden_truth or full_size or time_sweep or composition or alignment or store_policy" > gpurun_out/${EVID:-r06dlab}_tests_$v.log 2>&1
  echo "$v tests: $(tail -1 gpurun_out/${EVID:-r06dlab}_tests_$v.log)"
done
