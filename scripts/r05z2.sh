# Config 5: blocks of 2 and 1 waves (lib_var/jw2, jw1: each wave takes 2 / 4 candidate tiles in turn,
# so a wave's first tile's Jacobian stores overlap its next tile's sweep) against the 4-wave default;
# the config-5 parity tests with each variant, then the bench interleaved over 2 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z2
for v in jw2 jw1; do
  MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/$v/libmav_trajectory_generation.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "config5 or cost_at or sweep or jacobian" --timeout 120 --timeout-method thread > gpurun_out/r05z2/tests_$v.log 2>&1; rc=$?; echo "$v $(tail -1 gpurun_out/r05z2/tests_$v.log)"; [ $rc -le 1 ] || exit $rc
done
PATTERNS=generator EVID=r05z2 BENCHX="--workload config5" bash scripts/r05ab.sh jw2 jw1 || exit 1
