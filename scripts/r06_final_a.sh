# Round-6 closing run, part A: the -m gpu suite, smoke, and the bench lines --
# config 2 (the headline, default and the driver's 20/5), the config-3 shard, config 4, config 5,
# the off-pattern batches, the reference benchmark's long chains (K = 50 / 100, the long-chain DL
# kernel; K = 100 on the general kernel beside it), evaluateRange and the extrema.  The first crash or timeout ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06z}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR| passed| failed" $O/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
b() { f=$O/$1.json; shift; timeout -k 10 400 python bench.py "$@" > $f 2> $f.err || { tail $f.err; exit 1; }; }
b bench_c2
b bench_20_5 --steps 20 --warmup 5
b bench_c3 --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline
b bench_c4 --workload config4
b bench_c5 --workload config5
b bench_c2_accel --pattern accel-ends --no-cpu-baseline --no-end-to-end
b bench_c2_accel_column --pattern accel-ends --column-kernel --no-cpu-baseline --no-end-to-end
b bench_c2_vel --pattern interior-vel --no-cpu-baseline --no-end-to-end
b bench_c2_vel_column --pattern interior-vel --column-kernel --no-cpu-baseline --no-end-to-end
b bench_c4_accel --workload config4 --pattern accel-ends --no-cpu-baseline --no-end-to-end
b bench_c4_accel_column --workload config4 --pattern accel-ends --column-kernel --no-cpu-baseline --no-end-to-end
b bench_k50 --segments 50 --no-cpu-baseline --no-end-to-end
b bench_k100 --segments 100 --steps 200 --no-cpu-baseline --no-end-to-end
b bench_k100_general --segments 100 --steps 50 --warmup 20 --general-kernel --no-cpu-baseline --no-end-to-end
timeout -k 10 200 python scripts/bench_eval.py > $O/bench_eval.json 2> $O/bench_eval.err || { tail $O/bench_eval.err; exit 1; }
timeout -k 10 200 python scripts/bench_extrema.py > $O/bench_extrema.json 2> $O/bench_extrema.err || { tail $O/bench_extrema.err; exit 1; }
timeout -k 10 300 python scripts/bench_dlx_shapes.py > $O/bench_dlx_shapes.jsonl 2> $O/bench_dlx_shapes.err || { tail $O/bench_dlx_shapes.err; exit 1; }
timeout -k 10 300 python scripts/timing_eval.py > $O/latency_table.jsonl 2> $O/latency_table.err || { tail $O/latency_table.err; exit 1; }
for f in bench_c2 bench_20_5 bench_c3 bench_c4 bench_c5 bench_c2_accel bench_c2_accel_column bench_c2_vel bench_c2_vel_column bench_c4_accel bench_c4_accel_column bench_k50 bench_k100 bench_k100_general; do
  python -c "import json; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"
done
cat $O/bench_dlx_shapes.jsonl
echo OK > $O/done
