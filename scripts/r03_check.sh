# Round-3 GPU check: every -m gpu test, smoke(), and the bench as the driver runs it (20/5) next to
# the default (500/200) to check the time-based warmup.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_20_5.json 2> gpurun_out/bench_20_5.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
timeout -k 10 300 python scripts/bench_eval.py > gpurun_out/bench_eval.json 2> gpurun_out/bench_eval.err || exit $?
timeout -k 10 300 python scripts/bench_extrema.py > gpurun_out/bench_extrema.json 2> gpurun_out/bench_extrema.err || exit $?
