# Round 6: the bench lines alone on the final build (after the profiles whose captures they quote as
# roofline.traffic): config 2, the config-3 shard, config 4, config 5, the off-pattern batches and the
# long chains.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06j}
mkdir -p $O
export TMPDIR=/tmp
b() { f=$O/$1.json; shift; timeout -k 10 400 python bench.py "$@" > $f 2> $f.err || { tail $f.err; exit 1; }; }
b bench_c2
b bench_c3 --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline
b bench_c4 --workload config4
b bench_c5 --workload config5
b bench_c2_accel --pattern accel-ends --no-cpu-baseline --no-end-to-end
b bench_c2_vel --pattern interior-vel --no-cpu-baseline --no-end-to-end
b bench_c4_accel --workload config4 --pattern accel-ends --no-cpu-baseline --no-end-to-end
b bench_k50 --segments 50 --no-cpu-baseline --no-end-to-end
b bench_k100 --segments 100 --steps 200 --no-cpu-baseline --no-end-to-end
for f in bench_c2 bench_c3 bench_c4 bench_c5 bench_c2_accel bench_c2_vel bench_c4_accel bench_k50 bench_k100; do
  python -c "import json; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'], 'traffic', r['traffic'])"
done
echo OK > $O/done
