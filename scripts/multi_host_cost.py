#!/usr/bin/env python3
"""Host-side cost of N concurrent host-array pipelines, on the one-GPU box.

mtg_solve_linear_batch_multi with n contexts runs n host threads, each driving its context's chunk
pipeline (H2D, kernel, D2H; pageable arrays go through pinned bounce buffers, which costs host
memcpy).  With 8 GPUs that is 8 pipelines in one process under the box's CPU quota.  Here all n
contexts sit on the one device, so the PCIe link is shared and the wall rate is not an 8-GPU figure;
what this measures is the HOST work per trajectory (process CPU seconds, all threads) and whether it
grows when 8 pipelines run at once.  From it: the trajectories/s that the usable CPUs could feed,
the host-side ceiling of an 8-GPU node for host-array callers.

  python scripts/multi_host_cost.py [--per-ctx 125000] [--reps 3] > gpurun_out/multi_host_cost.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-ctx", type=int, default=125000, help="trajectories per context (config 3's shard)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--contexts", default="1,8")
    args = ap.parse_args()
    import ctypes
    import torch
    import bench
    import mav_trajectory_generation_cmake_amd as mtg
    from mav_trajectory_generation_cmake_amd import _native as nat
    from mav_trajectory_generation_cmake_amd.solver import _addr
    lib = nat.load()

    def multi(ctxs, v, m, t, out):
        # outputs preallocated and touched once (a fresh array per call would measure page faults)
        handles = (ctypes.c_void_p * len(ctxs))(*[c.handle for c in ctxs])
        nat.check(lib.mtg_solve_linear_batch_multi(ctypes.cast(handles, ctypes.c_void_p), len(ctxs), 10, 3, 10, 4,
                                                   len(v), _addr(v), _addr(m), _addr(t), _addr(out), None, None,
                                                   None, None, 0), ctxs[0].handle)
    host = bench.host_cpu_info()
    S = args.per_ctx
    v1, m1, t1 = mtg.random_vertices_path_batch(10, 3, 10, S, seed0=0)
    for n in [int(x) for x in args.contexts.split(",")]:
        B = n * S
        vals = np.ascontiguousarray(np.tile(v1, (n, 1, 1, 1)))
        mask = np.ascontiguousarray(np.tile(m1, (n, 1)))
        times = np.ascontiguousarray(np.tile(t1, (n, 1)))
        ctxs = [mtg.Context(0) for _ in range(n)]
        try:
            for mode in ("pageable", "pinned"):
                if mode == "pinned":
                    v, m, t = (torch.from_numpy(x).pin_memory().numpy() for x in (vals, mask, times))
                    out = torch.zeros((B, 10, 3, 10), dtype=torch.float64).pin_memory().numpy()
                else:
                    v, m, t = vals, mask, times
                    out = np.zeros((B, 10, 3, 10))
                multi(ctxs, v, m, t, out)  # warm: buffers, threads
                walls, cpus = [], []
                for _ in range(args.reps):
                    c0, w0 = time.process_time(), time.perf_counter()
                    multi(ctxs, v, m, t, out)
                    walls.append(time.perf_counter() - w0)
                    cpus.append(time.process_time() - c0)
                wall, cpu = float(np.median(walls)), float(np.median(cpus))
                cpu_per_traj = cpu / B
                rec = {"contexts": n, "mode": mode, "batch": B, "wall_s": wall, "traj_per_s_wall": B / wall,
                       "cpu_s": cpu, "cpu_us_per_traj": cpu_per_traj * 1e6,
                       "cpu_cores_busy": cpu / wall,
                       "host_feed_ceiling_traj_per_s": host["usable_cpus"] / cpu_per_traj,
                       "usable_cpus": host["usable_cpus"], "note": "all contexts on device 0 (shared PCIe link)"}
                print(json.dumps(rec), flush=True)
        finally:
            for c in ctxs:
                c.close()


if __name__ == "__main__":
    main()
