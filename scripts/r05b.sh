# Round-5: the -m gpu suite on the current build, then config 2 and the off-pattern batches on the
# default library and on variant libraries given as arguments (scripts/variant_lib.sh), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r05b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR| passed| failed" $O/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
lib() { [ "$1" = default ] && echo mav_trajectory_generation_cmake_amd/lib/libmav_trajectory_generation.so || echo mav_trajectory_generation_cmake_amd/lib_var/$1/libmav_trajectory_generation.so; }
for r in 1 2; do
  for v in default "$@"; do
    for p in ${PATTERNS:-generator accel-ends interior-vel}; do
      f=$O/bench_${v}_${p}_$r.json
      MTG_LIBRARY=$(lib $v) timeout -k 10 200 python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-end-to-end --pattern $p $BENCHX > $f 2> $f.err || { tail $f.err; exit 1; }
      python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$v $p', r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"
    done
  done
done
echo OK > $O/done
