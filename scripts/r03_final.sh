# Round-3 closing evidence on the final build: every -m gpu test and smoke(), bench lines (configs
# 2, 4, 5, config 3's per-GPU shard, the driver's 20/5 run), evaluateRange and extrema benches, and
# the rocprofv3 kernel-trace summaries of the config-2 and config-4 bench commands.  Each step
# time-limited; the first failure ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
for W in config2 config4 config5; do
  timeout -k 10 400 python bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || { tail $O/bench_$W.err; exit 1; }
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 300 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
timeout -k 10 200 python scripts/bench_eval.py > $O/bench_eval.json 2> $O/bench_eval.err || exit 1
timeout -k 10 200 python scripts/bench_extrema.py > $O/bench_extrema.json 2> $O/bench_extrema.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o run -- \
    python3 bench.py --no-cpu-baseline > $O/bench_c2_trace.json 2> $O/bench_c2_trace.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o run -- \
    python3 bench.py --workload config4 --no-cpu-baseline > $O/bench_c4_trace.json 2> $O/bench_c4_trace.err || exit 1
echo OK > $O/done
