# A/B of evaluateRange variant libraries (scripts/variant_lib.sh with UNITS=mtg_eval): bit-exact
# tests, then scripts/bench_eval.py, interleaved over 2 rounds.  usage: bash scripts/eval_ab.sh NAME ...
# (NAME "default" is the main build in mav_trajectory_generation_cmake_amd/lib)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=mav_trajectory_generation_cmake_amd/lib_var
lib() { [ "$1" = default ] && echo mav_trajectory_generation_cmake_amd/lib/libmav_trajectory_generation.so || echo $L/$1/libmav_trajectory_generation.so; }
for v in $( [ -z "$NOPARITY" ] && echo "$@" ); do  # (NOPARITY=1: timing only, e.g. diagnostic builds)
  MTG_LIBRARY=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "evaluate or min_max" --timeout 120 --timeout-method thread > gpurun_out/evab_t.log 2>&1 || { tail -20 gpurun_out/evab_t.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/evab_t.log)"
done
for r in 1 2; do lib() { [ "$1" = default ] && echo mav_trajectory_generation_cmake_amd/lib/libmav_trajectory_generation.so || echo $L/$1/libmav_trajectory_generation.so; }
for v in "$@"; do
  NOCHECK=$NOPARITY MTG_LIBRARY=$(lib $v) timeout -k 10 120 python scripts/bench_eval.py > gpurun_out/evab_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/evab_$v.json').read().strip().splitlines()[-1]); print('$v', 'full_call_gpu_ms %.4f' % d['full_call_gpu_ms'], 'count_ms %.4f' % d['two_call']['count_ms_wall'], 'eval_gpu_ms %.4f' % d['two_call']['eval_gpu_ms'])"
done; done
