# Round-3 (second session) evidence on the final build: every -m gpu test and smoke(), bench lines
# for config 2 (column kernel by default at B = 1e4), config 3's per-GPU shard (DL kernel by default
# at B = 125000) and its column-kernel A/B, the driver's 20/5 run; rocprofv3 kernel trace + calibrated
# HBM counters and SQ counters of the config-3 shard.  Each step time-limited; the first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 300 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
timeout -k 10 300 python bench.py --batch 125000 --steps 100 --warmup 50 --no-cpu-baseline --column-kernel > $O/bench_c3_column.json 2> $O/bench_c3_column.err || exit 1
bash scripts/profile.sh 125000 "" _c3dl || exit $?
bash scripts/pmc_sq.sh 125000 sq_c3dl || exit $?
python3 scripts/pmc_summary.py gpurun_out/sq_c3dl_b125000 solve_dl > $O/sq_c3dl.txt 2>&1
echo OK > $O/done
