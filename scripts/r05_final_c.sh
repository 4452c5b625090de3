# Round-5 closing run, part C (the final build: long chains' forward sweep on register inputs and
# padded staging rows): part A (suite, smoke, bench lines), then rocprofv3 traces + calibrated HBM
# counters of config 2 and config 4, SQ counters of config 4, and a trace of an all-off-pattern
# batch (ends fixed to ACCELERATION) on the default path and on the column kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${EVID:-r05r}
EVID=$T bash scripts/r05_final_a.sh || exit $?
bash scripts/profile.sh 10000 "--no-end-to-end" _c2$T || exit $?
bash scripts/profile.sh 10000 "--workload config4 --no-end-to-end" _c4$T || exit $?
bash scripts/pmc_sq.sh 10000 sq_c4$T "--workload config4 --no-end-to-end" || exit $?
for v in default column; do
  x=""; [ $v = column ] && x="--column-kernel"
  OUT=gpurun_out/prof_accel_${v}$T; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
      python3 bench.py --no-cpu-baseline --no-end-to-end --pattern accel-ends $x > $OUT/bench.log 2>&1 || exit $?
done
echo OK > gpurun_out/prof_done_$T
