# Same-box A/B of library builds: bench each library (MTG_LIBRARY) interleaved, 3 rounds.
# usage: bash scripts/ab_libs.sh BATCH libdirA libdirB ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=$1; shift
for round in 1 2 3; do
  for L in "$@"; do
    MTG_LIBRARY=$L/libmav_trajectory_generation.so timeout -k 10 120 python bench.py --steps 40 --warmup 5 --batch $B --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit $?
    grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('%-40s B=%d kern_ms=%.4f min=%.4f value=%.4g' % ('$L', d['config']['batch_per_gpu'], r['kernel_ms'], r['kernel_ms_isolated_min'], d['value']))"
  done
done
