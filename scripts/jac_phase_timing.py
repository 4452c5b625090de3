#!/usr/bin/env python3
"""Per-phase cycle stamps of time_jacobian_kernel (config 5; debug build: make -C ... timing).

Run: MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so python scripts/jac_phase_timing.py
Each wave's lane 0 writes its s_memtime stamps (entry, staged, W formed, sweep done, stored) over
cost[b0][8 wave .. 8 wave + 4]; this prints the phase durations and the spread of entry times.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402

dev = torch.device("cuda", 0)
ctx = mtg.Context(0)
N, r, K, C = 10, 4, 10, 64
B = int(os.environ.get("B", "10000"))
vals, mask, times = mtg.random_vertices_path_batch(N, 3, K, B, seed0=0)
xf = np.random.default_rng(0).standard_normal((B, K + 1, N // 2, 3))
scales = np.repeat((0.5 + np.arange(C) / (C - 1.0))[:, None], K, axis=1)
x_d = torch.from_numpy(xf).to(dev)
t_d = torch.from_numpy(times).to(dev)
s_d = torch.from_numpy(np.ascontiguousarray(scales)).to(dev)
c_d = torch.empty((B, C), dtype=torch.float64, device=dev)
j_d = torch.empty((B, C, K), dtype=torch.float64, device=dev)
for jac, name in ((None, "cost"), (j_d, "cost+jac")):
    step = ctx.jacobian_call(N, r, x_d, t_d, s_d, c_d, jac, increment_time=0.0)
    for _ in range(30):
        step()
    torch.cuda.synchronize()
    st = c_d.cpu().numpy()[::16, :64].reshape(-1, 4, 16)[:, :, :5].reshape(-1, 5)  # [blocks*4 waves][5]
    t0 = st[:, 0].min()
    d = np.diff(st, axis=1)
    print("%s B=%d waves=%d  span %.0f cycles (first entry -> last stamp)" % (name, B, len(st), st[:, 4].max() - t0))
    q = np.percentile(st[:, 0] - t0, [10, 50, 90, 100])
    print("  entry offset   p10 %7.0f p50 %7.0f p90 %7.0f max %7.0f" % tuple(q))
    for i, n in enumerate(["staging", "W formed", "sweep", "stores"]):
        print("  %-13s mean %7.0f p10 %7.0f p90 %7.0f" % (n, d[:, i].mean(), np.percentile(d[:, i], 10),
                                                         np.percentile(d[:, i], 90)))
    print("  wave total    mean %7.0f" % (st[:, 4] - st[:, 0]).mean(), flush=True)
ctx.reset_stream()
