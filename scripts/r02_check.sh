# Round-2 GPU check: new GPU tests, then the bench at config 2 (1e4) and config 3's per-GPU shard
# (125000), each step under its own time limit; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_pytest.log 2>&1 || { tail -30 gpurun_out/r02_pytest.log; exit 1; }
tail -3 gpurun_out/r02_pytest.log
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/r02_bench_b10000.json 2> gpurun_out/r02_bench_b10000.err || { tail -20 gpurun_out/r02_bench_b10000.err; exit 1; }
timeout -k 10 300 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline > gpurun_out/r02_bench_b125000.json 2> gpurun_out/r02_bench_b125000.err || { tail -20 gpurun_out/r02_bench_b125000.err; exit 1; }
echo OK
