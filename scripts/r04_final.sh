# Round-4 closing check on the final build: the full -m gpu suite, smoke, the config-2 bench line,
# the evaluateRange bench line, and the DL kernel's SQ counters at config 2 (scripts/pmc_sq.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR| passed| failed" $O/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
timeout -k 10 200 python scripts/bench_eval.py > $O/bench_eval.json 2> $O/bench_eval.err || { tail $O/bench_eval.err; exit 1; }
bash scripts/pmc_sq.sh 10000 r04z_sq || exit $?
echo OK > $O/done
