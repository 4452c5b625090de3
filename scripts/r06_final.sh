# Round-6 closing run on the final build: part A (the -m gpu suite, smoke, every bench line,
# evaluateRange, extrema), then the profiles (scripts/r06_prof.sh: rocprof traces + calibrated HBM
# counters of every bench line, SQ counters of configs 2 and 4).  The first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${EVID:-r06f}
EVID=$T bash scripts/r06_final_a.sh || exit $?
EVID=${T}p bash scripts/r06_prof.sh || exit $?
