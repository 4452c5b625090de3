# Round 6 debugging: the N = 12 ends-pass tests on variant libraries (MTG_LIBRARY)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K="dl_ends_pass_n12 or (time_sweep_off_pattern and 12) or (general_masks_vs and 12-3-20-3)"
for v in "$@"; do
  echo "== $v"
  MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/$v/libmav_trajectory_generation.so timeout -k 10 300 \
    python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "$K" 2>&1 | tail -3
done
