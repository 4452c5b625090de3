# Round-2 closing evidence: bench lines (configs 2, 4, 5, config 3's per-GPU shard, evaluateRange)
# and the rocprofv3 kernel-trace summary of the config-2 bench command; each step time-limited.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
export TMPDIR=/tmp
O=gpurun_out/final
for W in config2 config4 config5; do
  timeout -k 10 400 python bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || { tail $O/bench_$W.err; exit 1; }
done
timeout -k 10 300 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
timeout -k 10 200 python scripts/bench_eval.py > $O/bench_eval.json 2> $O/bench_eval.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o run -- \
    python3 bench.py --no-cpu-baseline > $O/bench_c2_trace.json 2> $O/bench_c2_trace.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o run -- \
    python3 bench.py --workload config4 --no-cpu-baseline > $O/bench_c4_trace.json 2> $O/bench_c4_trace.err || exit 1
echo OK
