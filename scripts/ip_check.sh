# IP lane kernel + extrema kernel: parity tests, then config 2 at B = 1e4 and the config-3 shard (IP vs
# default), and the extrema bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "ip or min_max" --timeout 300 --timeout-method thread > gpurun_out/pytest_ip.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_ip.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_extrema.py > gpurun_out/bench_extrema.json 2> gpurun_out/bench_extrema.err || exit $?
for B in 10000 125000; do
  for k in "" "--ip-kernel"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --batch $B $k > gpurun_out/ipb_${B}${k}.json 2>/dev/null || exit $?
  done
done
