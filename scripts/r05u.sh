# evaluateRange diagnostics: the producer / consumer kernel and the one-wave kernel with every store
# dropped (compute alone), against both with stores; timing only.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05u
NOPARITY=1 bash scripts/eval_ab.sh default evpc0 pcns ns1 > gpurun_out/r05u/eval_ab.log 2>&1; rc=$?; cat gpurun_out/r05u/eval_ab.log; exit $rc
