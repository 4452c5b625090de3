# Round 6: the driver's short run (--steps 20 --warmup 5) with the runtime's default completion
# signalling and with HSA_ENABLE_INTERRUPT=0 (the host polls the completion signal instead of
# sleeping on an interrupt), interleaved, 3 rounds: wall time per step vs GPU time per step.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06sync}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in default poll; do
    f=$O/bench_${v}_$r.json
    if [ $v = poll ]; then export HSA_ENABLE_INTERRUPT=0; else unset HSA_ENABLE_INTERRUPT; fi
    timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-end-to-end > $f 2> $f.err || { tail $f.err; exit 1; }
    python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$v', 'ms_per_step %.4f' % (d['ms_per_step']*1e3), 'kernel_ms %.4f' % (r['kernel_ms']*1e3), 'iso %.4f' % (r['kernel_ms_isolated']*1e3), 'value %.4g' % d['value'])"
  done
done
echo OK > $O/done
