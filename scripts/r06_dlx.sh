# Round 6: the long-chain dimension-lane kernel (mtg_solve_dlx.inc) -- its parity tests, then bench
# lines for the reference benchmark's long chains (N = 10, K = 50 / 100, 1e4 trajectories) and a
# rocprof kernel trace of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06dlx}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dlx.py -m gpu -x -v --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > $O/pytest_dlx.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR| passed| failed|PASSED|FAILED|Error" $O/pytest_dlx.log | tail -60
[ $rc -eq 0 ] || { grep -B5 -A40 "^E  " $O/pytest_dlx.log | head -120; exit $rc; }
b() { f=$O/$1.json; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end "$@" > $f 2> $f.err || { tail $f.err; exit 1; }; }
for K in 20 50 100; do b bench_k$K --segments $K --steps 100 --warmup 50; done
for K in 20 50 100; do python -c "import json; d=json.load(open('$O/bench_k$K.json')); r=d['roofline']; print($K, '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --segments 100 --steps 50 --warmup 20 --no-cpu-baseline --no-end-to-end > $O/prof_k100.log 2>&1 || exit 1
rm -f $O/prof/run_kernel_trace.csv
head -5 $O/prof/run_kernel_stats.csv
echo OK > $O/done
