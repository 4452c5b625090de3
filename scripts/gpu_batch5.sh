set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "magnitude" > gpurun_out/ext_tests.log 2>&1 || exit $?
timeout -k 10 200 python scripts/bench_extrema.py > gpurun_out/bench_extrema.json 2>gpurun_out/bench_extrema.err || exit $?
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ext_trace -o run -- python3 scripts/bench_extrema.py > gpurun_out/ext_trace.log 2>&1
