# GPU parity tests, then A/B bench of the default (register-resident) and general kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for B in 10000 125000; do
  for K in "" "--general-kernel"; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --batch $B --no-cpu-baseline $K > gpurun_out/ab_b$B$K.log 2>&1 || exit $?
    grep '^{' gpurun_out/ab_b$B$K.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('B=%d %s value=%.4g kern_ms=%.4f frac=%.3f' % (d['config']['batch_per_gpu'], r['kernel'], d['value'], r['kernel_ms'], r['frac']))"
  done
done
