# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (scripts/micro/hbm_calib), then the
# round's rocprofv3 evidence for the bench kernels (scripts/profile.sh).  One PMC group per pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/calib
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/$c -o run -- ./scripts/micro/hbm_calib > $OUT/$c.log 2>&1 || exit $?
done
bash scripts/profile.sh 10000 "" _r02 || exit $?
bash scripts/profile.sh 10000 "--workload config4" _r02c4 || exit $?
bash scripts/profile.sh 125000 "--split" _r02split || exit $?
echo calib done
