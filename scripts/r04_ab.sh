# Round-4 DL-kernel A/B: the full -m gpu suite on the main build (failures reported, the run goes on
# unless the step crashed or timed out), then the DL kernel's time vs batch for the variant
# libraries (scripts/variant_lib.sh) interleaved over 2 rounds, then the bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r04c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR| passed| failed" $O/pytest_gpu.log | tail -30
[ $rc -le 1 ] || { echo "pytest rc=$rc"; tail -30 $O/pytest_gpu.log; exit $rc; }
NOPARITY=1 KERNELS=dl BATCHES="${BATCHES:-1024 10000 125000}" timeout -k 10 600 bash scripts/var_ab.sh ${VARIANTS:-main} > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
timeout -k 10 400 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
timeout -k 10 400 python bench.py --workload config4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 1; }
timeout -k 10 400 python bench.py --workload config4 --no-cpu-baseline --column-kernel > $O/bench_c4_column.json 2> $O/bench_c4_column.err || { tail $O/bench_c4_column.err; exit 1; }
for f in bench_c2 bench_c3 bench_c4 bench_c4_column; do python -c "import json,sys; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"; done
echo OK > $O/done
