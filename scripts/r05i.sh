# Round-5 measurements: host cost of 8 concurrent host-array pipelines (spinning vs sleeping waits),
# the host single-solve latency (C++ drop-in vs the oracle, one core), and the config-5, extrema and
# evaluateRange bench lines, with the box's counter list for the MFMA counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 300 python scripts/multi_host_cost.py --contexts 1,8 > $O/multi_host_spin.jsonl 2> $O/multi_host_spin.err || { tail $O/multi_host_spin.err; exit 1; }
MTG_HOST_WAIT=block timeout -k 10 300 python scripts/multi_host_cost.py --contexts 1,8 > $O/multi_host_block.jsonl 2> $O/multi_host_block.err || { tail $O/multi_host_block.err; exit 1; }
cat $O/multi_host_spin.jsonl $O/multi_host_block.jsonl
timeout -k 10 300 bash scripts/latency_cpp.sh > $O/latency_cpp.jsonl 2> $O/latency_cpp.err || { tail $O/latency_cpp.err; exit 1; }
cat $O/latency_cpp.jsonl
timeout -k 10 300 python bench.py --workload config5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail $O/bench_c5.err; exit 1; }
timeout -k 10 200 python scripts/bench_extrema.py > $O/bench_extrema.json 2> $O/bench_extrema.err || { tail $O/bench_extrema.err; exit 1; }
timeout -k 10 200 python scripts/bench_eval.py > $O/bench_eval.json 2> $O/bench_eval.err || { tail $O/bench_eval.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c5.json')); r=d['roofline']; print('c5', '%.4g' % d['value'], r['kernel'], 'kernel_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'])"
tail -1 $O/bench_extrema.json; tail -1 $O/bench_eval.json
echo OK > $O/done
