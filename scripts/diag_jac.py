#!/usr/bin/env python3
"""Kernel time of mtg_time_jacobian_batch (config 5) with and without the Jacobian output, at a few
batch sizes (diagnostics for the matrix-core sweep)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402

dev = torch.device("cuda", 0)
ctx = mtg.Context(0)
N, r, K, C = 10, 4, 10, 64
for B in (2000, 10000, 40000):
    vals, mask, times = mtg.random_vertices_path_batch(N, 3, K, B, seed0=0)
    sol = ctx.solve_linear_batch(N, r, vals, mask, times, free=True)
    xf = mtg.full_vertex_values(vals, mask, sol["free"], N)
    scales = np.repeat((0.5 + np.arange(C) / (C - 1.0))[:, None], K, axis=1)
    x_d = torch.from_numpy(xf).to(dev)
    t_d = torch.from_numpy(times).to(dev)
    s_d = torch.from_numpy(np.ascontiguousarray(scales)).to(dev)
    c_d = torch.empty((B, C), dtype=torch.float64, device=dev)
    j_d = torch.empty((B, C, K), dtype=torch.float64, device=dev)
    for name, jac, dlt in (("cost", None, 0.0), ("cost+jac", j_d, 0.0), ("cost+fd", j_d, 0.1)):
        step = ctx.jacobian_call(N, r, x_d, t_d, s_d, c_d, jac, increment_time=dlt)
        ctx.enable_timing(20)
        for _ in range(25):
            step()
        torch.cuda.synchronize()
        ms = float(np.mean(ctx.kernel_times_ms(20)))
        print("B=%6d %-9s kernel %.4f ms" % (B, name, ms), flush=True)
    ctx.reset_stream()
