# Config-4 DL kernel check: the N = 12 and DL tests, the config-4 bench line and its timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r04f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "${PYK:-n12 or cfg4 or config4 or golden or dl_ or composition or not_spd}" > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR| passed| failed" $O/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --workload config4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
for f in bench_c4 bench_c2; do python -c "import json,sys; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"; done
L=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so
MTG_LIBRARY=$L B=10000 N=12 K=20 timeout -k 10 120 python scripts/dl_timeline.py > $O/timeline.jsonl 2> $O/timeline.err || { tail $O/timeline.err; exit 1; }
cat $O/timeline.jsonl
