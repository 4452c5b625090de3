# Kernel iteration on the GPU box: GPU parity suite, then kernel time vs batch for config 2 and the
# config-4 line (each step under its own time limit; stops at the first failure).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/k_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/k_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/k_pytest.log | head -30; exit $rc; fi
fi
for B in ${BATCHES:-1024 8192 10000 131072}; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 100 --batch $B --no-cpu-baseline $EXTRA > gpurun_out/k_b$B.json 2> gpurun_out/k_b$B.err || { tail gpurun_out/k_b$B.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/k_b$B.json')); r=d['roofline']; print('B=$B value=%.4g kern_ms=%.4f frac=%.3f' % (d['value'], r['kernel_ms'], r['frac']))"
done
if [ -z "$NOC4" ]; then
timeout -k 10 120 python bench.py --workload config4 --steps 200 --warmup 100 --no-cpu-baseline > gpurun_out/k_c4.json 2> gpurun_out/k_c4.err || { tail gpurun_out/k_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/k_c4.json')); r=d['roofline']; print('config4 value=%.4g kern_ms=%.4f frac=%.3f' % (d['value'], r['kernel_ms'], r['frac']))"
fi
