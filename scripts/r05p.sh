# Config 4: the long chains' forward sweep on register-resident inputs as they land (lib_var/freg,
# with the padded staging rows) against lib_var/spad (padded rows, inputs parked before the sweep)
# and the main build: DL parity tests with the variant, then the bench interleaved over 2 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/${EVID:-r05p}
MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/${TESTV:-freg}/libmav_trajectory_generation.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "n12 or cfg4 or config4 or golden or dl or composition or not_spd" --timeout 120 --timeout-method thread > gpurun_out/${EVID:-r05p}/tests.log 2>&1; rc=$?; tail -2 gpurun_out/${EVID:-r05p}/tests.log; [ $rc -le 1 ] || exit $rc
PATTERNS=generator EVID=${EVID:-r05p} BENCHX="--workload config4" bash scripts/r05ab.sh ${VARIANTS:-spad freg} || exit 1
