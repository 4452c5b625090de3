# Round-end evidence: GPU tests, the three bench lines, rocprofv3 kernel stats + PMC traffic per
# workload (scripts/profile.sh), evaluateRange bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_round.sh > gpurun_out/round.log 2>&1 || { tail -20 gpurun_out/round.log; exit 1; }
tail -6 gpurun_out/round.log | cut -c1-400
bash scripts/profile.sh 10000 "" _c2 || exit $?
bash scripts/profile.sh 10000 "--workload config4" _c4 || exit $?
bash scripts/profile.sh 10000 "--workload config5" _c5 || exit $?
bash scripts/profile.sh 131072 "" _c2 || exit $?
echo profiles done
