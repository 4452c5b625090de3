# Round-4 evidence: -m gpu suite, then rocprofv3 kernel traces + calibrated HBM counters (one PMC
# pass per group) of the DL kernel at config 2, config 3's shard and config 4, and SQ counters at
# config 2 and config 4.  Each step time-limited; the first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r04d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR| passed| failed" $O/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
bash scripts/profile.sh 10000 "" _c2${EVID:-r04d} || exit $?
bash scripts/profile.sh 125000 "--steps 100 --warmup 50" _c3${EVID:-r04d} || exit $?
bash scripts/profile.sh 10000 "--workload config4" _c4${EVID:-r04d} || exit $?
if [ -z "$NOSQ" ]; then
  bash scripts/pmc_sq.sh 10000 sq_c2${EVID:-r04d} || exit $?
  bash scripts/pmc_sq.sh 10000 sq_c4${EVID:-r04d} "--workload config4" || exit $?
fi
echo OK > $O/done
