#!/usr/bin/env python3
"""Per-phase cycle counts of the lane-per-chain solve kernel (debug build with MTG_PHASE_TIMING).

Run: MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so \
     B=8192 python scripts/lane_phase_timing.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (share torch's HIP runtime)
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402

B = int(os.environ.get("B", "8192"))
vals, mask, times = mtg.random_vertices_path_batch(10, 3, 10, B, seed0=0)
ctx = mtg.Context(0)
for _ in range(3):
    out = ctx.solve_linear_batch(10, 4, vals, mask, times, free=True, lane=True)
f = out["free"].reshape(B, -1)[:, :5]
names = ["staging", "forward", "merge", "backward", "epilogue"]
tot = f.sum(axis=1)
print("B=%d lane kernel, s_memtime ticks per wave (mean over trajectories)" % B)
for i, n in enumerate(names):
    print("  %-9s mean %8.0f  p10 %8.0f  p90 %8.0f  (%.0f%%)" % (n, f[:, i].mean(), np.percentile(f[:, i], 10),
                                                             np.percentile(f[:, i], 90),
                                                             100 * f[:, i].mean() / tot.mean()))
print("  total     mean %8.0f" % tot.mean())
