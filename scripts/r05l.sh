# A/B of the pivot-minimum materialisation (default) against round 4's (pm0) at configs 2, 3 and 4
# and the off-pattern batches, with the DL parity tests on the default build first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05l
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "dl or golden or config4 or batch_composition or not_spd" --timeout 120 --timeout-method thread > gpurun_out/r05l/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r05l/tests.log; [ $rc -le 1 ] || exit $rc
PATTERNS="generator accel-ends interior-vel" EVID=r05l bash scripts/r05ab.sh pm0 || exit 1
PATTERNS=generator EVID=r05l3 BENCHX="--batch 125000" STEPS=100 bash scripts/r05ab.sh pm0 || exit 1
PATTERNS=generator EVID=r05l4 BENCHX="--workload config4" bash scripts/r05ab.sh pm0 || exit 1
