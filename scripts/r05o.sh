# Config 4: staging rows padded to an odd number of 16-B units (lib_var/spad) against the unpadded
# main build: the DL parity tests with the variant first, then the bench interleaved over 2 rounds,
# and the variant's LDS counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05o
MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/spad/libmav_trajectory_generation.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "n12 or cfg4 or config4 or golden" --timeout 120 --timeout-method thread > gpurun_out/r05o/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05o/tests.log; [ $rc -le 1 ] || exit $rc
PATTERNS=generator EVID=r05o BENCHX="--workload config4" bash scripts/r05ab.sh spad || exit 1
OUT=gpurun_out/sq_c4spad_b10000; mkdir -p $OUT
MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/spad/libmav_trajectory_generation.so timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $OUT/p1 -o run -- python3 bench.py --steps 10 --warmup 2 --batch 10000 --no-cpu-baseline --workload config4 --no-end-to-end > $OUT/p1.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $OUT solve_dl_kernel 2>/dev/null | head -8
