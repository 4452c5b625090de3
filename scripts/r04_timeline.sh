# DL kernel per-wave phase timeline (debug build lib_timing/, cmake -DMTG_PHASE_TIMING=ON)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r04e}
mkdir -p $O
L=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so
for B in 1024 10000 125000; do
  MTG_LIBRARY=$L B=$B timeout -k 10 120 python scripts/dl_timeline.py >> $O/timeline.jsonl 2> $O/timeline.err || { tail $O/timeline.err; exit 1; }
done
MTG_LIBRARY=$L B=10000 N=12 K=20 timeout -k 10 120 python scripts/dl_timeline.py >> $O/timeline.jsonl 2> $O/timeline.err || { tail $O/timeline.err; exit 1; }
cat $O/timeline.jsonl
