# SQ stall/instruction counters for the solve kernel (one PMC pass per group, kernel-trace only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=${1:-125000}
TAG=${2:-sq}
EXTRA=${3:-}
OUT=gpurun_out/${TAG}_b$B
mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS" \
           "SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT" \
           "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --steps 10 --warmup 2 --batch $B --no-cpu-baseline $EXTRA > $OUT/p$i.log 2>&1 || exit $?
done
# LDS / scalar / instruction-issue detail (second set)
for grp in "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM_NORM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --steps 10 --warmup 2 --batch $B --no-cpu-baseline $EXTRA > $OUT/p$i.log 2>&1 || { echo "group $grp failed"; }
done
rm -f $OUT/p*/run_kernel_trace.csv
