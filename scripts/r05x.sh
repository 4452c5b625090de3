# evaluateRange: the producer / consumer kernel with flag hand-over over 3 and 4 slots (lib_var/pcf3,
# pcf4) against the barrier-per-block default; bit-exact tests for all, bench_eval interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/${EVO:-r05x}
bash scripts/eval_ab.sh ${EVV:-default pcf3 pcf4} > gpurun_out/${EVO:-r05x}/eval_ab.log 2>&1; rc=$?; cat gpurun_out/${EVO:-r05x}/eval_ab.log; exit $rc
