# evaluateRange: the producer / consumer sample kernel (default) against the one-wave kernel
# (lib_var/evpc0); bit-exact tests for both, bench_eval interleaved over 2 rounds, and a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05t
bash scripts/eval_ab.sh default evpc0 > gpurun_out/r05t/eval_ab.log 2>&1; rc=$?; cat gpurun_out/r05t/eval_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05t/trace -o run -- python3 scripts/bench_eval.py > gpurun_out/r05t/bench_eval.log 2>&1 || exit $?
grep -E "eval_" gpurun_out/r05t/trace/run_kernel_stats.csv | cut -c1-60,200-260
