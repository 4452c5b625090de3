# parity suite, then the register kernel's phase split and kernel time vs batch (default path)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/p.log 2>&1
rc=$?
tail -2 gpurun_out/p.log
if [ $rc -ne 0 ]; then grep -E "^E " gpurun_out/p.log | head -20; exit $rc; fi
B=8192 MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so timeout -k 10 120 python scripts/phase_timing.py || exit $?
for B in 8192 10000 131072; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --batch $B --no-cpu-baseline > gpurun_out/s.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/s.json')); r=d['roofline']; print('B=$B kern_ms=%.4f frac=%.3f' % (r['kernel_ms'], r['frac']))"
done
