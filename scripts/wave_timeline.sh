set -o pipefail
mkdir -p gpurun_out
export MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so
for B in ${BATCHES:-1024 8192 10000 16384}; do
  B=$B timeout -k 10 120 python scripts/wave_timeline.py >> gpurun_out/wave_timeline.jsonl || exit $?
done
