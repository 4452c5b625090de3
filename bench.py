#!/usr/bin/env python3
"""Benchmark: trajectories/s of the batched 10-segment N=10 3-D minimum-snap solve.

Default workload (BASELINE.json configs[1], "config 2"): per GPU a batch of B = 1e4
trajectories from the reference bench generator
createRandomVerticesPath(3, 10, 5.0, SNAP, seed) + estimateSegmentTimes(2, 2, 6.5)
(src/polynomial_timing_evaluation.cpp:34-112), seeds rank*B .. rank*B+B-1 (so
at N = 8 with --batch 125000 this is exactly config 3's 1e6 sharded batch).
One step = one batched setupFromVertices + solveLinear of the whole batch
(fused HIP kernel, inputs already resident in HBM, coefficients written to HBM).

Other workloads (--workload), each its own JSON line:
  config4  N=12, K=20, r=JERK: createRandomVertices(SNAP, 20, [-10,-20,-10], [10,20,10], seed)
           + estimateSegmentTimes(3, 5) (src/vertex.cpp:27-79, :162-178)
  config5  the config-2 problems, solved once (untimed), then one step = the cost of the solved
           derivatives and its segment-time Jacobian at 64 candidate time allocations
           (getCostAndGradientDerivative + getCostAndGradientTime's J_d gradient at T_c = s_c T,
           s_c = 0.5 + c/63; mtg_time_jacobian_batch, v_mfma_f64_16x16x4_f64)

Multi-GPU: one process per GPU, contiguous shards, no data-path collective ("scaling": "weak");
a barrier + MAX-over-ranks of the timed region.  Under torch.distributed.run the launcher's
WORLD_SIZE must equal --gpus; without one, `bench.py --gpus N` starts the N rank processes itself
(self_launch) before anything touches the GPU.

Prints ONE JSON line (rank 0).  Also reports the dominant kernel's roofline
(algorithmic bytes / measured kernel time vs 8 TB/s HBM peak) and the CPU
baseline (the oracle restatement of the reference algorithm on host cores).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
C5_CANDIDATES = 64


def algorithmic_bytes_per_traj(N, D, K):
    """Bytes the ABI must move per trajectory: values [V][h][D] f64 + mask [V] u8
    + times [K] f64 in, coefficients [K][D][N] f64 out.  Config 2: 1411 + 2400 = 3811 B."""
    V, h = K + 1, N // 2
    return V * h * D * 8 + V + K * 8 + K * D * N * 8


def cost_sweep_bytes_per_traj(N, D, K, C):
    """mtg_time_jacobian_batch: vertex derivatives [V][h][D] + times [K] in, costs [C] and the time
    Jacobian [C][K] out (config 5: 1320 + 80 + 512 + 5120 = 7032 B; the candidate scales [C][K] are
    shared by the batch)."""
    V, h = K + 1, N // 2
    return V * h * D * 8 + K * 8 + C * 8 + C * K * 8


def shard_seed0(rank, batch_per_rank):
    """Rank r solves trajectories with seeds r*B .. r*B+B-1: contiguous shards of one global
    batch of world*B independent problems (no data-path exchange)."""
    return rank * batch_per_rank


def max_over_ranks(x, dist):
    """Slowest rank's elapsed time (the job's wall clock); identity at world size 1.  A host-side
    MAX over the gloo group (the only cross-rank step is this scalar)."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def csrc_digest():
    """SHA-256 over the kernel sources (mav_trajectory_generation_cmake_amd/csrc, names and contents):
    the build identity a PMC capture is valid for."""
    import hashlib
    d = os.path.join(ROOT, "mav_trajectory_generation_cmake_amd", "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".inc", ".h", ".cpp", ".py")):
            h.update(f.encode())
            with open(os.path.join(d, f), "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()


def traffic_key(kernel_prefix, workload, pattern="generator"):
    """profiles/pmc_traffic.json key of a capture: kernel, bench workload and vertex pattern."""
    return "%s|%s|%s" % (kernel_prefix, workload, pattern)


def traffic_from_profiles(kernel_prefix, batch, workload, pattern="generator"):
    """HBM bytes per launch of the kernel from the committed PMC summary (profiles/), and where they
    come from: (bytes, source) or (None, reason).  A capture is used only for the same kernel, workload,
    vertex pattern and batch, taken on a build of the same kernel sources (csrc_digest) -- otherwise
    the line carries traffic null (scripts/summarize_profiles.py writes the captures)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, "no profiles/pmc_traffic.json"
    try:
        with open(path) as f:
            d = json.load(f)
        ent = d.get(traffic_key(kernel_prefix, workload, pattern), {}).get(str(batch))
        if ent is None:
            return None, "no PMC capture of %s for this workload / pattern / batch" % kernel_prefix
        if ent.get("csrc_sha256") != csrc_digest():
            return None, "the PMC capture (%s) is of other kernel sources" % ent.get("profile")
        return float(ent["hbm_bytes_per_launch"]), ent.get("profile")
    except Exception as e:  # (a malformed summary is not a measurement)
        return None, "unreadable pmc_traffic.json: %s" % e


def _oracle_lib():
    from oracle import pyoracle
    lib = pyoracle.build(build_dir="_build_bench", arch=os.environ.get("MTG_ORACLE_ARCH", "native"))
    pyoracle._LIB = None
    pyoracle.lib(lib)  # the copy built on this host with -march=native
    return pyoracle


def cpu_baseline(values, mask, times, N, r, target_s, threads):
    """Oracle (faithful C restatement of lin_impl, dense QR in place of SparseQR) on host cores."""
    pyoracle = _oracle_lib()
    m32 = mask.astype(np.uint32)
    done = 0
    t0 = time.perf_counter()
    while True:
        pyoracle.solve_linear_batch(N, r, values, m32, times, threads=threads)
        done += len(values)
        el = time.perf_counter() - t0
        if el >= target_s:
            break
    return done / el, el, done


def cpu_baseline_cost(xfull, times, scales, N, r, target_s, threads):
    """Oracle getCostAndGradientDerivative at candidate times with getCostAndGradientTime's J_d
    gradient, as the reference computes it: per candidate the reference's per-segment H (A, Schur
    A^-1, Q) and d^T R d, and per segment the central difference with increment_time 0.1."""
    pyoracle = _oracle_lib()
    done = 0
    t0 = time.perf_counter()
    while True:
        pyoracle.cost_time_jacobian_batch(N, r, xfull, times, scales, 0.1, threads=threads)
        done += len(xfull) * len(scales)
        el = time.perf_counter() - t0
        if el >= target_s:
            break
    return done / el, el, done


def host_cpu_info():
    """The host's CPUs as this process sees them: nproc (os.cpu_count), the affinity mask, the cgroup
    CPU quota (cpu.max), the lscpu model name; usable_cpus = the cores the process can actually run
    on at once (affinity, capped by the quota) -- the CPU baseline uses all of them."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity_cpus"] = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(p)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    try:
        import subprocess
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in txt.splitlines():
            if line.startswith("Model name:"):
                info["lscpu_model"] = line.split(":", 1)[1].strip()
            elif line.startswith("Socket(s):") or line.startswith("Core(s) per socket:") or \
                    line.startswith("Thread(s) per core:"):
                info[line.split(":", 1)[0].strip().lower().replace("(s)", "s").replace(" ", "_")] = \
                    line.split(":", 1)[1].strip()
    except Exception:
        pass
    usable = info["affinity_cpus"] or 1
    if quota:
        usable = max(1, min(usable, int(quota)))
    info["usable_cpus"] = usable
    return info


def end_to_end(ctx, N, r, values, mask, times, unit, h2d_bytes, d2h_bytes, n=30):
    """Host arrays in and out through the C ABI (not `value`): H2D, kernels, D2H and the
    synchronisation of a caller whose batch lives in host memory.  Batches above 8 MB run as the
    library's chunk pipeline; measured from pageable numpy arrays (staged through the runtime) and
    from pinned arrays (torch pin_memory, DMA'd in place), the two interleaved call by call over n
    calls each, reported as the median with the 10th / 90th percentiles."""
    import torch
    B, V, h, D = values.shape
    K = V - 1
    res = {"unit": unit, "h2d_bytes_per_traj": h2d_bytes, "d2h_bytes_per_traj": d2h_bytes, "calls": n}
    pinned_in = [torch.from_numpy(x).pin_memory().numpy() for x in (values, mask, times)]
    pinned_out = torch.empty((B, K, D, N), dtype=torch.float64).pin_memory().numpy()
    page_out = np.empty((B, K, D, N))
    modes = (("pageable", (values, mask, times), page_out), ("pinned", pinned_in, pinned_out))
    for _ in range(3):
        for _, (v, m, t), o in modes:
            ctx.solve_linear_batch(N, r, v, m, t, coeffs=o)
    secs = {name: [] for name, _, _ in modes}
    for _ in range(n):
        for name, (v, m, t), o in modes:
            t0 = time.perf_counter()
            ctx.solve_linear_batch(N, r, v, m, t, coeffs=o)
            secs[name].append(time.perf_counter() - t0)
    for name, _, _ in modes:
        x = np.array(secs[name])
        med = float(np.median(x))
        res[name] = {"value": B / med, "ms_per_call_median": med * 1e3,
                     "ms_per_call_p10": float(np.percentile(x, 10)) * 1e3,
                     "ms_per_call_p90": float(np.percentile(x, 90)) * 1e3,
                     "pcie_gbs": B * (h2d_bytes + d2h_bytes) / med / 1e9}
    res["value"] = res["pinned"]["value"]
    res["note"] = ("per GPU; host arrays in/out, synchronous; median over interleaved calls; chunks pipelined "
                   "over 4 slots above 8 MB (H2D / kernel / D2H of consecutive chunks overlap; D2H issued by "
                   "the context's persistent worker thread on the GPU's NUMA node)")
    return res


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_envs(n, port, base_env=None):
    """The environment of each of the n ranks a self-launched `bench.py --gpus n` starts: what
    torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_*),
    rendezvous on 127.0.0.1."""
    base = dict(os.environ if base_env is None else base_env)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def self_launch(n, argv, cmd=None, popen=None):
    """`bench.py --gpus n` without an outer launcher: start n rank processes (this script again, same
    arguments) and wait for them.  Called before anything touches the GPU -- this process imports
    neither torch nor the library -- so the children are started from a process with no HIP state.
    Rank 0's JSON line reaches stdout through the inherited descriptor.  If any rank fails the others
    are stopped and the first failing exit code is returned."""
    import subprocess
    if popen is None:
        popen = subprocess.Popen
    if cmd is None:
        cmd = [sys.executable, os.path.abspath(__file__)]
    procs = [popen(cmd + list(argv), env=e) for e in rank_envs(n, _free_port())]
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:
                    q.kill()
        if pending:
            time.sleep(0.05)
    return rc


PATTERNS = {
    "generator": "the reference generators' vertex pattern (ends fix derivatives 0..4, interior vertices "
                 "their position)",
    "accel-ends": "off-pattern: createRandomVertices(ACCELERATION, K, [-50]^3, [50]^3, seed) + "
                  "estimateSegmentTimes(3, 5): ends fix derivatives 0..2 only (the reference's "
                  "2_vertices_rand pattern, test/test_polynomial_optimization.cpp:747-774)",
    "interior-vel": "off-pattern: the workload's problems with every interior vertex also fixing its "
                    "velocity (to 0: a stop-and-go waypoint path)",
}


def make_problems(workload, N, K, B, seed0, pattern="generator"):
    import mav_trajectory_generation_cmake_amd as mtg
    if pattern == "accel-ends":
        return mtg.random_vertices_batch(N, 3, K, B, [-50.0] * 3, [50.0] * 3, seed0=seed0, max_derivative=2,
                                         v_max=3.0, a_max=5.0)
    if workload == "config4":
        values, mask, times = mtg.random_vertices_batch(N, 3, K, B, [-10.0, -20.0, -10.0], [10.0, 20.0, 10.0],
                                                        seed0=seed0, max_derivative=4, v_max=3.0, a_max=5.0)
    else:
        values, mask, times = mtg.random_vertices_path_batch(N, 3, K, B, seed0=seed0)
    if pattern == "interior-vel":
        mask = mask.copy()
        mask[:, 1:-1] |= 2
        values = values.copy()
        values[:, 1:-1, 1, :] = 0.0
    return values, mask, times


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: enough warmup for the GPU clocks to settle (a 10-launch warmup left the B = 131072
    # kernel at 195 us instead of 155 us), and a timed region of ~15 ms at config 2
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--min-warmup-ms", type=float, default=300.0,
                    help="keep warming up until this much wall time has passed, whatever --warmup is (the "
                         "GPU clocks settle over ~100 ms of back-to-back launches)")
    ap.add_argument("--workload", choices=["config2", "config4", "config5"], default="config2")
    ap.add_argument("--batch", type=int, default=10000, help="trajectories per GPU (configs 2, 4, 5: 1e4)")
    ap.add_argument("--pattern", choices=sorted(PATTERNS), default="generator",
                    help="vertex constraint pattern of the solve workloads (off-pattern A/B; not the headline)")
    ap.add_argument("--segments", type=int, default=None)
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--timing-stride", type=int, default=0,
                    help="also sample every n-th step's kernel with its own HIP event pair (0: none; the "
                         "sampled launches add event overhead to the timed region)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-sample", type=int, default=20000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-end-to-end", action="store_true",
                    help="skip the host-array leg (profiling runs: the trace then holds only the bench's own grid)")
    ap.add_argument("--split", action="store_true", help="two-kernel path (assembly + block Cholesky)")
    ap.add_argument("--general-kernel", action="store_true",
                    help="force the general LDS-resident fused kernel (A/B against the default)")
    ap.add_argument("--dl-kernel", action="store_true",
                    help="the dimension-lane kernel where it applies (A/B against the default)")
    ap.add_argument("--column-kernel", action="store_true",
                    help="the register column kernel where it applies, whatever the batch size (A/B)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:  # no outer launcher: one process per GPU, started from here
            sys.exit(self_launch(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks"
                 % (args.gpus, os.environ["WORLD_SIZE"]))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; (more ranks than GPUs, as in a rehearsal of the multi-rank path on a smaller
    # box, share them round-robin)
    ndev = torch.cuda.device_count()
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(ndev, 1)
    if world > 1:
        # gloo: the ranks exchange only a barrier and one scalar (no data-path collective), so the
        # multi-GPU run does not depend on RCCL
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import mav_trajectory_generation_cmake_amd as mtg

    wl = args.workload
    if wl == "config4":
        N, K, r = args.N or 12, args.segments or 20, 3
    else:
        N, K, r = args.N or 10, args.segments or 10, 4
    D = 3
    B = args.batch
    values, mask, times = make_problems(wl, N, K, B, shard_seed0(rank, B), args.pattern)
    v_d = torch.from_numpy(values).to(dev)
    m_d = torch.from_numpy(mask).to(dev)
    t_d = torch.from_numpy(times).to(dev)
    ctx = mtg.Context(local)
    # Kernel time (roofline): the HIP events g0 / g1 around the timed region on the launch stream;
    # the launches run back to back (rocprofv3 shows no gap between them), so region time / steps is
    # the kernel's steady-state duration.  Optionally (--timing-stride n) every n-th step goes through
    # a second context that carries an event pair in the dispatch packet; events cost ~4.5 us of GPU
    # time per launch at config 2 (scripts/host_overhead.py), charged to `value`, so this is off by
    # default.  After the region, launches that each carry their own event pair give the duration of
    # a launch that does not overlap its predecessor (reported as kernel_ms_isolated).
    ctx_t = mtg.Context(local)
    stream = torch.cuda.current_stream(dev)
    if wl == "config5":
        # solve once (untimed) for the free derivatives, then time the candidate-cost sweep
        sol = ctx.solve_linear_batch(N, r, values, mask, times, free=True)
        xfull = mtg.full_vertex_values(values, mask, sol["free"], N)
        scales = np.repeat((0.5 + np.arange(C5_CANDIDATES) / (C5_CANDIDATES - 1.0))[:, None], K, axis=1)
        x_d = torch.from_numpy(xfull).to(dev)
        s_d = torch.from_numpy(np.ascontiguousarray(scales)).to(dev)
        out_d = torch.empty((B, C5_CANDIDATES), dtype=torch.float64, device=dev)
        jac_d = torch.empty((B, C5_CANDIDATES, K), dtype=torch.float64, device=dev)
        step = ctx.jacobian_call(N, r, x_d, t_d, s_d, out_d, jac_d)
        step_t = ctx_t.jacobian_call(N, r, x_d, t_d, s_d, out_d, jac_d)
        kname = "time_jacobian_kernel"
    else:
        out_d = torch.empty((B, K, D, N), dtype=torch.float64, device=dev)
        # one step = one launch of the solve on torch's current stream
        kw = dict(split=args.split, general=args.general_kernel, dl=args.dl_kernel, column=args.column_kernel)
        step = ctx.solve_call(N, r, v_d, m_d, t_d, out_d, **kw)
        step_t = ctx_t.solve_call(N, r, v_d, m_d, t_d, out_d, **kw)
        nat = mtg._native
        kflags = ((nat.MTG_FLAG_SPLIT_KERNELS if args.split else 0) | (nat.MTG_FLAG_GENERAL_KERNEL if args.general_kernel else 0)
                  | (nat.MTG_FLAG_DL_KERNEL if args.dl_kernel else 0) | (nat.MTG_FLAG_COLUMN_KERNEL if args.column_kernel else 0))
        kname = mtg._native.solve_kernel(N, D, K, r, kflags, B=B)
    stride = args.timing_stride
    timed_steps = [i for i in range(args.steps) if stride > 0 and i % stride == 0]
    ctx.enable_timing(0)
    ctx_t.enable_timing(max(len(timed_steps), 1))
    plan = [step_t if stride > 0 and i % stride == 0 else step for i in range(args.steps)]

    # warmup: at least --warmup steps AND at least --min-warmup-ms of wall time
    w0 = time.perf_counter()
    warm = 0
    while warm < args.warmup or (time.perf_counter() - w0) * 1e3 < args.min_warmup_ms:
        for _ in range(max(1, min(args.warmup, 100))):
            step()
            warm += 1
        torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    g0 = torch.cuda.Event(enable_timing=True)
    g1 = torch.cuda.Event(enable_timing=True)
    # (the start event is enqueued before the wall clock starts: its host-side record costs ~14 us,
    # which is the measuring apparatus's, not the workload's -- 0.7 us per step of the driver's
    # 20-step region, profiles/r06/ab/r06t0.json; the GPU-side kernel_ms is the same either way)
    g0.record(stream)
    t0 = time.perf_counter()
    for fn in plan:
        fn()
    g1.record(stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    per_launch = ctx_t.kernel_times_ms(len(timed_steps)) if timed_steps else np.zeros(0)
    gpu_ms = g0.elapsed_time(g1)
    kern_ms = gpu_ms / args.steps
    # (A sampled launch's own event interval inside the region starts while its predecessor is still
    # draining, so it reads longer than the per-step time: config 2, 20.1 vs 18.8 us.)
    n_iso = 32
    ctx_t.enable_timing(n_iso)
    for _ in range(n_iso):
        step_t()
    torch.cuda.synchronize(dev)
    iso = ctx_t.kernel_times_ms(n_iso)
    el = max_over_ranks(el, dist if world > 1 else None)

    # spot check of the timed outputs (finite) -- not timed
    assert np.isfinite(out_d.cpu().numpy()).all(), "non-finite outputs"
    if wl == "config5":
        assert np.isfinite(jac_d.cpu().numpy()).all(), "non-finite Jacobian"

    if wl == "config5":
        units = B * C5_CANDIDATES
        bpt = cost_sweep_bytes_per_traj(N, D, K, C5_CANDIDATES)
        metric = ("trajectory-candidate cost+time-Jacobian evaluations/sec "
                  "(config 5: 64 time allocations x 10-seg N=10 3-D)")
        unit = "candidate evaluations/s"
        workload = ("config5: %d x 64 candidate allocations (K=%d, N=%d, D=%d, r=SNAP) per GPU, d fixed; "
                    "cost [B][64] + dJ/dT [B][64][K] (exact) on the matrix cores" % (B, K, N, D))
        data = ("synthetic: config-2 problems (createRandomVerticesPath + estimateSegmentTimes(2,2,6.5)) solved once; "
                "candidates T_c = (0.5 + c/63) T")
    else:
        units = B
        bpt = algorithmic_bytes_per_traj(N, D, K)
        if wl == "config4":
            metric = "trajectories/sec (config 4: 20-seg, N=12, 3-D min-jerk)"
            workload = "config4: %d x (K=%d, N=%d, D=%d, r=JERK) per GPU, device-resident" % (B, K, N, D)
            data = ("synthetic: createRandomVertices(SNAP,20,[-10,-20,-10],[10,20,10],seed) "
                    "+ estimateSegmentTimes(3,5), seeds rank*B..rank*B+B-1")
        else:
            metric = "trajectories/sec (10-seg, N=10, 3-D min-snap) at 1/2/4/8 MI355X"
            workload = "config2: %d x (K=%d, N=%d, D=%d, r=SNAP) per GPU, device-resident" % (B, K, N, D)
            data = ("synthetic: reference bench generator createRandomVerticesPath(3,10,5.0,SNAP,seed) "
                    "+ estimateSegmentTimes(2,2,6.5), seeds rank*B..rank*B+B-1")
        unit = "trajectories/s"
        if args.pattern != "generator":
            workload += "; pattern %s" % args.pattern
            data = "synthetic, " + PATTERNS[args.pattern]
    total = units * world * args.steps
    value = total / el
    achieved = bpt * B / (kern_ms * 1e-3) / 1e9
    # (a capture is keyed by the workload's shape: "config2-K100" for config 2's generator at K = 100)
    wl_key = wl if (args.N is None and args.segments is None) else "%s-N%dK%d" % (wl, N, K)
    traffic, traffic_src = traffic_from_profiles(kname, B, wl_key, args.pattern)
    out = {
        "metric": metric,
        "value": value,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_steps_run": warm,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": data,
        "config": {"workload": workload, "batch_per_gpu": B, "global_batch": B * world, "segments": K, "N": N,
                   "D": D, "derivative_to_optimize": r, "parallelism": "shard%d" % world, "kernel_path": kname},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": kname,
                     "kernel_ms": kern_ms,
                     "kernel_ms_method": "HIP events around the timed region on the launch stream / steps "
                     "(back-to-back launches)",
                     "kernel_ms_isolated": float(np.mean(iso)), "kernel_ms_isolated_min": float(np.min(iso)),
                     "kernel_ms_sampled": float(np.mean(per_launch)) if len(per_launch) else None,
                     "kernel_launches_sampled": len(per_launch), "gpu_ms_timed_region": gpu_ms,
                     "algorithmic_bytes_per_traj": bpt},
        "cpu_baseline": None,
    }
    # end-to-end (not `value`): host arrays in and out through the C ABI's staging -- H2D, kernel,
    # D2H, synchronize -- the PCIe-inclusive rate of a caller that holds its batch in host memory
    if wl != "config5" and not args.no_end_to_end:
        out["end_to_end"] = end_to_end(ctx, N, r, values, mask, times, unit, bpt - K * D * N * 8, K * D * N * 8)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # (the CPU baseline is an N = 1 figure)
        host = host_cpu_info()
        threads = int(os.environ.get("MTG_CPU_THREADS", host["usable_cpus"]))
        S = min(args.cpu_sample, B)
        if wl == "config5":
            S = min(S, 1000)
            rate, cel, done = cpu_baseline_cost(xfull[:S], times[:S], scales, N, r, args.cpu_seconds, threads)
            sample = ("%d trajectories x %d candidates of this rank's shard, evaluated repeatedly for %.1f s "
                      "(%d candidate cost+Jacobian evaluations; the Jacobian as the reference forms it, a "
                      "central difference per segment) by the oracle restatement (-O3 -march=native, OpenMP)"
                      % (S, C5_CANDIDATES, cel, done))
        else:
            rate, cel, done = cpu_baseline(values[:S], mask[:S], times[:S], N, r, args.cpu_seconds, threads)
            sample = ("%d trajectories of this rank's shard, solved repeatedly for %.1f s "
                      "(%d solves) by the oracle restatement (-O3 -march=native, OpenMP)" % (S, cel, done))
        out["cpu_baseline"] = {"value": rate, "unit": unit, "cores": threads, "kind": "port", "sample": sample,
                               "host": host}
    ctx.close()
    ctx_t.close()
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
