# Round 6: where the reference benchmark's long chains (N=10, K=50 / 100) stand on the batched path --
# bench lines (1e4 trajectories per launch) for K = 20, 50, 100 and the latency table.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r06long}
mkdir -p $O
export TMPDIR=/tmp
b() { f=$O/$1.json; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end "$@" > $f 2> $f.err || { tail $f.err; exit 1; }; }
for K in 20 50 100; do b bench_k$K --segments $K --steps 100 --warmup 50; done
for K in 20 50 100; do python -c "import json; d=json.load(open('$O/bench_k$K.json')); r=d['roofline']; print($K, '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"; done
timeout -k 10 300 python scripts/timing_eval.py > $O/latency_table.jsonl 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency_table.jsonl
echo OK > $O/done
