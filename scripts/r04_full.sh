# Round-4 check: the full -m gpu suite, smoke, bench lines for configs 2, 3 (shard), 4 and the
# 20/5 driver run, and the DL timeline at config 2.  Failures of tests are reported; the run goes on
# unless a step crashed or timed out.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r04h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR| passed| failed" $O/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || { tail $O/bench_20_5.err; exit 1; }
timeout -k 10 400 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
timeout -k 10 400 python bench.py --workload config4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 1; }
for f in bench_c2 bench_20_5 bench_c3 bench_c4; do python -c "import json,sys; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"; done
L=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so
for B in 10000 125000; do
  MTG_LIBRARY=$L B=$B timeout -k 10 120 python scripts/dl_timeline.py >> $O/timeline.jsonl 2> $O/timeline.err || { tail $O/timeline.err; exit 1; }
done
cat $O/timeline.jsonl
echo OK > $O/done
