# Round-3 (second session) bench lines on the final build: config 2 (DL kernel by default at
# B = 1e4) and its column-kernel A/B, the driver's 20/5 run, config 3's per-GPU shard and its
# column-kernel A/B, config 4 and config 5.  Each step time-limited; the first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --column-kernel > $O/bench_c2_column.json 2> $O/bench_c2_column.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 300 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
timeout -k 10 300 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline --column-kernel > $O/bench_c3_column.json 2> $O/bench_c3_column.err || exit 1
for W in config4 config5; do
  timeout -k 10 400 python bench.py --workload $W --no-cpu-baseline > $O/bench_$W.json 2> $O/bench_$W.err || exit 1
done
echo OK > $O/bench_done
