set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for pad in 0 8192 16384 32768; do
  MTG_DEBUG_LDS_PAD=$pad timeout -k 10 120 python bench.py --steps 20 --warmup 3 --batch 125000 --no-cpu-baseline > gpurun_out/occ_$pad.log 2>&1 || exit $?
done
