# GPU tests, then one bench line per workload (config 2 default, 4, 5) with CPU baselines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E " gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
for W in config2 config4 config5; do
  timeout -k 10 400 python bench.py --workload $W > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$W.json')); r=d['roofline']; c=d['cpu_baseline']; print('$W value=%.4g %s kern_ms=%.4f frac=%.3f cpu=%.4g' % (d['value'], d['unit'], r['kernel_ms'], r['frac'], c['value']))"
done
