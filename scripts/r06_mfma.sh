# Round 6: MFMA counters of the config-5 kernel on the final build (as r05_final_b.sh), and the
# store-policy bit-equality test.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${EVID:-r06m}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "store_policy" > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/mfma_c5${T}_b10000
mkdir -p $OUT
i=0
for grp in "SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" \
           "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/p$i.log 2>&1 || exit $?
  rm -f $OUT/p$i/run_kernel_trace.csv
done
echo OK > gpurun_out/${T}_done
