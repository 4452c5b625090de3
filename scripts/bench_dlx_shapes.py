#!/usr/bin/env python3
"""Long-chain shapes: per-launch time of the default path (the long-chain DL kernel +
its rest kernel) against the general kernel, 1e4 device-resident trajectories of the bench generator
(createRandomVerticesPath, ends fixed up to min(4, N/2 - 1)), HIP events around 20 back-to-back
launches after a warm-up.  One JSON line per shape."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402
from mav_trajectory_generation_cmake_amd import _native as nat  # noqa: E402

B = 10000
dev = torch.device("cuda", 0)
ctx = mtg.Context(0)
for (N, D, K, r) in [(10, 3, 50, 4), (10, 3, 100, 4), (12, 3, 40, 3), (8, 3, 50, 3), (6, 3, 50, 2), (10, 3, 20, 4)]:
    vals, mask, times = mtg.random_vertices_path_batch(N, D, K, B, seed0=1, max_derivative=min(4, N // 2 - 1))
    v, m, t = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (vals, mask, times))
    out = torch.empty((B, K, D, N), dtype=torch.float64, device=dev)
    line = {"N": N, "D": D, "K": K, "r": r, "B": B}
    for name, kw in (("default", {}), ("general", {"general": True})):
        step = ctx.solve_call(N, r, v, m, t, out, **kw)
        for _ in range(10):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20 if name == "default" else 5
        e0.record()
        for _ in range(n):
            step()
        e1.record()
        torch.cuda.synchronize()
        line[name + "_us"] = round(e0.elapsed_time(e1) / n * 1e3, 2)
        line[name + "_kernel"] = nat.solve_kernel(N, D, K, r, nat.MTG_FLAG_GENERAL_KERNEL if kw else 0, B=B)
    alg = B * ((K + 1) * (N // 2) * D * 8 + (K + 1) + K * 8 + K * D * N * 8)
    line["algorithmic_MB"] = round(alg / 1e6, 1)
    line["frac_default"] = round(alg / (line["default_us"] * 1e-6) / 8e12, 3)
    line["speedup"] = round(line["general_us"] / line["default_us"], 2)
    print(json.dumps(line), flush=True)
