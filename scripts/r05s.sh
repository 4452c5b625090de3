# evaluateRange: rocprofv3 kernel trace of scripts/bench_eval.py (per-kernel durations of the one-call
# path: clock + counts, scan, the stored-run sample kernel, the rest launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05s; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/bench_eval.py > $OUT/bench_eval.log 2>&1 || exit $?
cut -c1-160 $OUT/trace/run_kernel_stats.csv
