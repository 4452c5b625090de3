# diagnostic: N = 12, r = 5 NOT_SPD on the long-chain DL kernel vs the general kernel
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, ".")
import numpy as np
import mav_trajectory_generation_cmake_amd as mtg
from mav_trajectory_generation_cmake_amd import random_vertices_path_batch
from _util import scale_normalised_error
ctx = mtg.Context(0)
for (N, D, K, r, B, seed) in [(12, 1, 25, 5, 437, 3100 + 25 + 1), (12, 3, 20, 5, 437, 3100 + 25 + 1)]:
    vals, mask, times = random_vertices_path_batch(N, D, K, B, seed0=seed, max_derivative=4)
    kw = dict(status=True, cost=True)
    x = ctx.solve_linear_batch(N, r, vals, mask, times, **kw)
    g = ctx.solve_linear_batch(N, r, vals, mask, times, general=True, **kw)
    bad = np.nonzero((x["status"] != 0) | (g["status"] != 0))[0]
    print(N, D, K, r, "x bad", np.nonzero(x["status"])[0], "g bad", np.nonzero(g["status"])[0])
    for b in bad[:3]:
        print("  b", b, "times", times[b].min(), times[b].max(), "x", x["status"][b], "g", g["status"][b],
              "cost", x["cost"][b], g["cost"][b],
              "dg", scale_normalised_error(x["coeffs"][b:b+1], g["coeffs"][b:b+1], times[b:b+1]))
