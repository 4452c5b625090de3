# Round 6: the driver's short run with the start event recorded before / after the wall clock
# starts (bench.py vs a copy recording it before t0, since adopted by bench.py), interleaved; then the self-launched two-rank bench on
# one GPU (both ranks share it: a rehearsal of the multi-rank path, not a scaling point).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06t0}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3 4; do
  for v in bench scripts/_bench_t0; do
    f=$O/$(basename $v)_$r.json
    timeout -k 10 200 python $v.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end > $f 2> $f.err || { tail $f.err; exit 1; }
    python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$v', 'ms_per_step %.3f' % (d['ms_per_step']*1e3), 'kernel_us %.3f' % (r['kernel_ms']*1e3), 'value %.4g' % d['value'])"
  done
done
timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 20 --no-cpu-baseline --no-end-to-end > $O/bench_gpus2.json 2> $O/bench_gpus2.err || { tail $O/bench_gpus2.err; exit 1; }
cat $O/bench_gpus2.json | cut -c1-300
echo OK > $O/done
