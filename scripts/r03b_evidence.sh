# Round-3 (second session) evidence on the final build: every -m gpu test and smoke(); rocprofv3
# kernel trace + calibrated HBM counters and SQ counters of the DL kernel at config 2 (B = 1e4) and
# config 3's per-GPU shard (B = 125000).  Each step time-limited; the first failure ends it.
# (Bench lines: scripts/r03b_bench.sh, after scripts/summarize_profiles.py has merged the traffic.)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
bash scripts/profile.sh 10000 "" _c2dl || exit $?
bash scripts/profile.sh 125000 "" _c3dl || exit $?
bash scripts/pmc_sq.sh 10000 sq_c2dl || exit $?
python3 scripts/pmc_summary.py gpurun_out/sq_c2dl_b10000 solve_dl > $O/sq_c2dl.txt 2>&1
bash scripts/pmc_sq.sh 125000 sq_c3dl || exit $?
python3 scripts/pmc_summary.py gpurun_out/sq_c3dl_b125000 solve_dl > $O/sq_c3dl.txt 2>&1
echo OK > $O/done
