# Round-6 A/B (as r05ab.sh): the solve bench on the default library and variant libraries (scripts/variant_lib.sh),
# interleaved over 2 rounds, for the vertex patterns in $PATTERNS (bench.py --pattern) and the
# extra bench arguments in $BENCHX.  usage: bash scripts/r05ab.sh VARIANT ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06ab}
mkdir -p $O
export TMPDIR=/tmp
lib() { [ "$1" = default ] && echo mav_trajectory_generation_cmake_amd/lib/libmav_trajectory_generation.so || echo mav_trajectory_generation_cmake_amd/lib_var/$1/libmav_trajectory_generation.so; }
for r in 1 2; do
  for v in default "$@"; do
    for p in ${PATTERNS:-generator accel-ends interior-vel}; do
      f=$O/bench_${v}_${p}_$r.json
      MTG_LIBRARY=$(lib $v) timeout -k 10 200 python bench.py --steps ${STEPS:-200} --warmup 100 --no-cpu-baseline --no-end-to-end --pattern $p $BENCHX > $f 2> $f.err || { tail $f.err; exit 1; }
      python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$v $p', r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"
    done
  done
done
echo OK > $O/done
