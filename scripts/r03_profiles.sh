# Round-3 profile evidence: rocprofv3 kernel trace + calibrated HBM counters for config 2, config 4
# and config 3's per-GPU shard (B = 125000), SQ counters for config 4.  Each step time-limited.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/profile.sh 10000 "" _c2 || exit $?
bash scripts/profile.sh 10000 "--workload config4" _c4 || exit $?
bash scripts/profile.sh 125000 "" _c3 || exit $?
bash scripts/pmc_sq.sh 10000 sq_c4 "--workload config4" || exit $?
echo OK
