# Round 6: the DL kernel's coefficient-store cache policy (plain vs sc1, MTG_DL_STORE_SC1) against
# the batch size, config-2 and config-4 shapes, interleaved: where the sc1 stores stop paying.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06sc1}
mkdir -p $O
export TMPDIR=/tmp
run() {  # tag policy args...
  t=$1; p=$2; shift 2
  f=$O/${t}_sc$p.json
  MTG_DL_STORE_SC1=$p timeout -k 10 200 python bench.py --steps 100 --warmup 50 --no-cpu-baseline --no-end-to-end "$@" > $f 2> $f.err || { tail $f.err; exit 1; }
  python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$t sc1=$p', 'kernel_us %.2f' % (r['kernel_ms']*1e3), 'frac %.3f' % r['frac'])"
}
for B in ${BATCHES:-10000 20000 30000 40000 50000 70000 100000}; do
  for p in 0 1; do run c2_b$B $p --batch $B || exit 1; done
done
for B in ${BATCHES4:-10000 15000 20000 30000}; do
  for p in 0 1; do run c4_b$B $p --batch $B --workload config4 || exit 1; done
done
echo OK > $O/done
