set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
for W in config2 config4 config5; do
  timeout -k 10 400 python bench.py --workload $W > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || exit $?
  cat gpurun_out/bench_$W.json
done
timeout -k 10 200 python scripts/bench_eval.py > gpurun_out/bench_eval.json 2>&1 || exit $?
cat gpurun_out/bench_eval.json
