# Round-3 closing evidence on the final build (DL kernel with compile-time tables): every -m gpu test
# and smoke(), bench lines (configs 2, 4, 5, config 3's shard, the driver's 20/5 run, column-kernel
# A/Bs), rocprofv3 kernel trace + calibrated HBM counters of the DL kernel at configs 2 and 3's shard.
# Each step time-limited; the first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r03c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --column-kernel > $O/bench_c2_column.json 2> $O/bench_c2_column.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 300 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
timeout -k 10 300 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline --column-kernel > $O/bench_c3_column.json 2> $O/bench_c3_column.err || exit 1
bash scripts/profile.sh 10000 "" _c2dl${EVID:-f} || exit $?
bash scripts/profile.sh 125000 "" _c3dl${EVID:-f} || exit $?
echo OK > $O/done
