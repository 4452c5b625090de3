# one iteration of kernel work on the GPU box: parity tests, phase timing, bench at B=1e4 and 1.25e5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so timeout -k 10 300 python scripts/phase_timing.py || exit $?
for B in 10000 125000; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --batch $B --no-cpu-baseline > gpurun_out/iter_b$B.log 2>&1 || exit $?
  grep '^{' gpurun_out/iter_b$B.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('B=%d %s value=%.4g kern_ms=%.4f frac=%.3f' % (d['config']['batch_per_gpu'], r['kernel'], d['value'], r['kernel_ms'], r['frac']))"
done
