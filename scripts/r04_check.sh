# Round-4 check on the GPU box: every -m gpu test, smoke, the default bench line, the self-launched
# 2-rank bench (both ranks on the one device: a rehearsal of `bench.py --gpus 2`), the DL/column
# kernel sweep over batch sizes and the host cost of concurrent host-array pipelines.
# Each step time-limited; the first failure ends it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${EVID:-r04a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_gpus2.json 2> $O/bench_gpus2.err || { tail $O/bench_gpus2.err; exit 1; }
cat $O/bench_c2.json $O/bench_gpus2.json | cut -c1-300
if [ -n "$SWEEP" ]; then
  KERNELS=column,dl timeout -k 10 300 python scripts/sweep_kernels.py 1 10 64 256 640 1024 2048 4096 10000 125000 > $O/sweep.log 2>&1 || exit 1
  cat $O/sweep.log
fi
if [ -n "$HOSTCOST" ]; then
  timeout -k 10 600 python scripts/multi_host_cost.py > $O/multi_host_cost.jsonl 2> $O/multi_host_cost.err || { tail $O/multi_host_cost.err; exit 1; }
  cat $O/multi_host_cost.jsonl
fi
echo OK > $O/done
