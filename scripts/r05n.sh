# evaluateRange: the clock kernels with the segment times staged in LDS (default) against the
# previous build (lib_var/evord0: times read from global memory in the clock loop); bit-exact tests
# for both, then scripts/bench_eval.py interleaved over 2 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05n
bash scripts/eval_ab.sh default evord0 > gpurun_out/r05n/eval_ab.log 2>&1; rc=$?; cat gpurun_out/r05n/eval_ab.log; exit $rc
