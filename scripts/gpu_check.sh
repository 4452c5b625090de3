set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch 125000 --no-cpu-baseline > gpurun_out/bench_b125k.log 2>&1 || exit $?
bash scripts/profile.sh 10000 > gpurun_out/profile.log 2>&1
