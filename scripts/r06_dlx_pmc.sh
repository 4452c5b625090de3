# Round 6: HBM traffic of the long-chain DL kernel (N = 10, K = 20 / 50 / 100, 1e4 trajectories):
# separate FETCH_SIZE / WRITE_SIZE passes (MI355X guide's HBM section: 2 x FETCH + WRITE).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06dlxpmc}
mkdir -p $O
export TMPDIR=/tmp
for K in 20 50 100; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/k${K}_$C -o run -- \
      python3 bench.py --segments $K --steps 20 --warmup 20 --no-cpu-baseline --no-end-to-end > $O/k${K}_$C.log 2>&1 || exit 1
    rm -f $O/k${K}_$C/run_kernel_trace.csv
  done
  python3 -c "import json; d=json.load(open('$O/k${K}_FETCH_SIZE.log')); print($K, d['roofline']['kernel_ms'])" || true
done
echo OK > $O/done
