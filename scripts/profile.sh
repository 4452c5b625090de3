# rocprofv3 evidence for profiles/: kernel trace + stats, then one PMC pass per counter group
# (never --pmc together with trace domains other than --kernel-trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=${1:-10000}
EXTRA=${2:-}
TAG=${3:-}
OUT=gpurun_out/prof${TAG}_b$B
mkdir -p $OUT
run() { timeout -k 10 300 "$@"; }
run rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --batch $B --no-cpu-baseline $EXTRA > $OUT/bench_trace.log 2>&1 || exit $?
run rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 bench.py --steps 50 --warmup 200 --batch $B --no-cpu-baseline $EXTRA > $OUT/bench_fetch.log 2>&1 || exit $?
run rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
    python3 bench.py --steps 50 --warmup 200 --batch $B --no-cpu-baseline $EXTRA > $OUT/bench_write.log 2>&1 || exit $?
run rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_l2 -o run -- \
    python3 bench.py --steps 50 --warmup 200 --batch $B --no-cpu-baseline $EXTRA > $OUT/bench_l2.log 2>&1 || exit $?
# (the per-dispatch kernel traces are not summarised -- the stats and counter files are: dropped so a
# set of profiles fits gpurun_out)
rm -f $OUT/trace/run_kernel_trace.csv $OUT/pmc_*/run_kernel_trace.csv
