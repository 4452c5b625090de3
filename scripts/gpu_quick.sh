set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for B in 10000 125000; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --batch $B --no-cpu-baseline > gpurun_out/bench_b$B.log 2>&1 || exit $?
done
