# Round-6 profiles of the final build: rocprofv3 kernel traces + calibrated HBM counters
# (scripts/profile.sh: FETCH_SIZE, WRITE_SIZE, TCC hit/miss, one pass each) for every bench line that
# reports roofline.traffic -- config 2, the config-3 shard, config 4, config 5, and the off-pattern
# batches on the default path and the column kernel, the long chains K = 50 / 100 -- then SQ counters of config 2 and config 4.
# Summaries: scripts/summarize_profiles.py (WORKLOAD / PATTERN key the traffic).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${EVID:-r06p}
P=scripts/profile.sh
bash $P 10000 "--no-end-to-end" _c2$T || exit $?
bash $P 125000 "--no-end-to-end" _c3$T || exit $?
bash $P 10000 "--workload config4 --no-end-to-end" _c4$T || exit $?
bash $P 10000 "--workload config5" _c5$T || exit $?
bash $P 10000 "--pattern accel-ends --no-end-to-end" _acc$T || exit $?
bash $P 10000 "--pattern accel-ends --column-kernel --no-end-to-end" _acccol$T || exit $?
bash $P 10000 "--pattern interior-vel --no-end-to-end" _vel$T || exit $?
bash $P 10000 "--pattern interior-vel --column-kernel --no-end-to-end" _velcol$T || exit $?
bash $P 10000 "--workload config4 --pattern accel-ends --no-end-to-end" _c4acc$T || exit $?
bash $P 10000 "--no-end-to-end --column-kernel" _c2col$T || exit $?
bash $P 10000 "--segments 50 --no-end-to-end" _k50$T || exit $?
bash $P 10000 "--segments 100 --no-end-to-end" _k100$T || exit $?
bash scripts/pmc_sq.sh 10000 sq_c2$T "--no-end-to-end" || exit $?
bash scripts/pmc_sq.sh 10000 sq_c4$T "--workload config4 --no-end-to-end" || exit $?
echo OK > gpurun_out/prof_done_$T
