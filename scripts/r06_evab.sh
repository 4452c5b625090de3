# Round 6: evaluateRange A/B of variant libraries (scripts/bench_eval.py, interleaved), then the
# evaluateRange parity tests on each variant.  usage: bash scripts/r06_evab.sh VARIANT ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06evab}
mkdir -p $O
export TMPDIR=/tmp
lib() { [ "$1" = default ] && echo mav_trajectory_generation_cmake_amd/lib/libmav_trajectory_generation.so || echo mav_trajectory_generation_cmake_amd/lib_var/$1/libmav_trajectory_generation.so; }
for r in 1 2; do
  for v in default "$@"; do
    MTG_LIBRARY=$(lib $v) timeout -k 10 200 python scripts/bench_eval.py > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail $O/${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v', 'full %.4f ms' % d['full_call_gpu_ms'], 'count %.4f ms' % d['two_call']['count_ms_wall'])"
  done
done
for v in "$@"; do
  MTG_LIBRARY=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "evaluate_range" > $O/tests_$v.log 2>&1
  echo "$v tests: $(tail -1 $O/tests_$v.log)"
done
echo OK > $O/done
