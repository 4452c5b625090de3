export TMPDIR=/tmp; mkdir -p gpurun_out/r05k
MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_var/zpin/libmav_trajectory_generation.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "dl_general or dl_kernel or batch_composition" --timeout 120 --timeout-method thread > gpurun_out/r05k/zpin_tests.log 2>&1; tail -2 gpurun_out/r05k/zpin_tests.log
PATTERNS="accel-ends interior-vel" EVID=r05kz bash scripts/r05ab.sh zpin || exit 1
PATTERNS=generator EVID=r05k BENCHX="--workload config4" bash scripts/r05ab.sh nost12 || exit 1
PATTERNS=generator EVID=r05k5 BENCHX="--workload config5" bash scripts/r05ab.sh jold || exit 1
MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so timeout -k 10 120 python scripts/jac_phase_timing.py > gpurun_out/r05k/jac_phase.txt 2>&1; cat gpurun_out/r05k/jac_phase.txt
