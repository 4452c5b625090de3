# Round-5 first look: evaluateRange A/B of the pair-clock branch (lib_var/evpair), the config-2 bench
# on the current build, and the off-pattern regime (default vs column vs general kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
bash scripts/eval_ab.sh default evpair > $O/eval_ab.log 2>&1 || { tail -30 $O/eval_ab.log; exit 1; }
cat $O/eval_ab.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
for p in accel-ends interior-vel; do
  for k in "" --column-kernel --general-kernel; do
    timeout -k 10 200 python bench.py --steps 100 --warmup 50 --no-cpu-baseline --no-end-to-end --pattern $p $k > $O/bench_${p}${k}.json 2> $O/bench_${p}${k}.err || { tail $O/bench_${p}${k}.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${p}${k}.json')); r=d['roofline']; print('$p $k', r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'])"
  done
done
python -c "import json; d=json.load(open('$O/bench_c2.json')); r=d['roofline']; print('c2', '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"
echo OK > $O/done
