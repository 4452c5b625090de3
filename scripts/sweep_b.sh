# Kernel time of the default path vs batch size (single-wave latency vs throughput regime),
# plus the per-phase cycle split of the register kernel (debug build) at small and large B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 1024 4096 8192 10000 16384 32768 65536 131072; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --batch $B --no-cpu-baseline > gpurun_out/sweep_$B.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/sweep_$B.json')); r=d['roofline']; print('B=$B kern_ms=%.4f step_ms=%.4f frac=%.3f' % (r['kernel_ms'], d['ms_per_step'], r['frac']))"
done
for B in 8192 125000; do
  B=$B MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so timeout -k 10 120 python scripts/phase_timing.py || exit $?
done
