# IP kernel A/B, then the extrema kernel's counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/ip_check.sh || exit $?
bash scripts/pmc_extrema.sh || exit $?
