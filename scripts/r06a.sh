# Round 6, first GPU pass on the ends-pass build: the DL-kernel parity tests (ends / general-mask
# passes, full-size off-pattern batches, truth samples, time sweeps, batch composition), then bench
# lines for config 2, the off-pattern batches (default and column kernel), config 4 and the
# config-3 shard.  The first failure or timeout ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "dl_ or golden_truth or full_size or time_sweep or composition or kat" > $O/pytest_dl.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR| passed| failed|PASSED|FAILED" $O/pytest_dl.log | tail -80
[ $rc -eq 0 ] || exit $rc
b() { f=$O/$1.json; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end "$@" > $f 2> $f.err || { tail $f.err; exit 1; }; }
b bench_c2
b bench_c2_accel --pattern accel-ends
b bench_c2_accel_column --pattern accel-ends --column-kernel
b bench_c2_vel --pattern interior-vel
b bench_c2_vel_column --pattern interior-vel --column-kernel
b bench_c4 --workload config4
b bench_c4_accel --workload config4 --pattern accel-ends
b bench_c3 --batch 125000 --steps 100 --warmup 50
for f in bench_c2 bench_c2_accel bench_c2_accel_column bench_c2_vel bench_c2_vel_column bench_c4 bench_c4_accel bench_c3; do
  python -c "import json; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"
done
echo OK > $O/done
