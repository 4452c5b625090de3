# Validation of the long-chain pivot-minimum build and the longest-first evaluateRange order: the
# closing run's part A (suite, smoke, bench lines), the evaluateRange A/B against the build without
# the order (lib_var/evord0), then config 4's rocprof trace, HBM counters and SQ counters again
# (r05z's predate the pivot-minimum change).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
EVID=r05m bash scripts/r05_final_a.sh || exit $?
NOPARITY=1 bash scripts/eval_ab.sh default evord0 > gpurun_out/r05m/eval_ab.log 2>&1 || { cat gpurun_out/r05m/eval_ab.log; exit 1; }
cat gpurun_out/r05m/eval_ab.log
bash scripts/profile.sh 10000 "--workload config4 --no-end-to-end" _c4r05m || exit $?
bash scripts/pmc_sq.sh 10000 sq_c4r05m "--workload config4 --no-end-to-end" || exit $?
echo OK > gpurun_out/r05m/prof_done
