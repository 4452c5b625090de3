# diagnostic: N = 12, r = 5 -- which kernel agrees with 60-digit truth (DLX / DL / general / column)
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, ".")
import numpy as np
import mav_trajectory_generation_cmake_amd as mtg
from mav_trajectory_generation_cmake_amd import random_vertices_path_batch
from _util import scale_normalised_error as sne
from make_golden import truth_solve_banded
ctx = mtg.Context(0)
for (N, D, K, r) in [(12, 1, 21, 5), (12, 1, 20, 5), (12, 1, 21, 4), (10, 1, 13, 4), (10, 1, 13, 3), (12, 1, 6, 5)]:
    vals, mask, times = random_vertices_path_batch(N, D, K, 6, seed0=11, max_derivative=4)
    x = ctx.solve_linear_batch(N, r, vals, mask, times, status=True)
    g = ctx.solve_linear_batch(N, r, vals, mask, times, general=True, status=True)
    c = ctx.solve_linear_batch(N, r, vals, mask, times, column=True, status=True)
    for b in range(3):
        tr = truth_solve_banded(N, r, vals[b], mask[b], times[b])[None]
        sl = slice(b, b + 1)
        print(N, K, r, b, "default(%s)" % mtg._native.solve_kernel(N, D, K, r), "%.2e" % sne(x["coeffs"][sl], tr, times[sl]),
              "general %.2e" % sne(g["coeffs"][sl], tr, times[sl]), "column %.2e" % sne(c["coeffs"][sl], tr, times[sl]),
              x["status"][b], g["status"][b], flush=True)
