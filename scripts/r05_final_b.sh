# Round-5 closing run, part B (the final build): rocprofv3 kernel traces and calibrated HBM counters
# (one PMC pass per group) of the bench's own launches (--no-end-to-end: no other grid in the trace)
# for config 2, the config-3 shard, config 4 and config 5; SQ counters for configs 2 and 4; MFMA
# counters for config 5; SQ counters of the extrema kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${EVID:-r05z}
bash scripts/profile.sh 10000 "--no-end-to-end" _c2$T || exit $?
bash scripts/profile.sh 125000 "--steps 100 --warmup 50 --no-end-to-end" _c3$T || exit $?
bash scripts/profile.sh 10000 "--workload config4 --no-end-to-end" _c4$T || exit $?
bash scripts/profile.sh 10000 "--workload config5" _c5$T || exit $?
bash scripts/pmc_sq.sh 10000 sq_c2$T "--no-end-to-end" || exit $?
bash scripts/pmc_sq.sh 10000 sq_c4$T "--workload config4 --no-end-to-end" || exit $?
OUT=gpurun_out/mfma_c5${T}_b10000
mkdir -p $OUT
i=0
for grp in "SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" \
           "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/p$i.log 2>&1 || exit $?
done
bash scripts/pmc_extrema.sh || exit $?
echo OK > gpurun_out/prof_done_$T
