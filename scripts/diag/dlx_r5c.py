# diagnostic: the test batch (N = 12, D = 1, K = 25, r = 5): DLX vs general vs truth on the worst pairs
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "tests/golden"); sys.path.insert(0, ".")
import numpy as np
import mav_trajectory_generation_cmake_amd as mtg
from mav_trajectory_generation_cmake_amd import random_vertices_path_batch
from _util import scale_normalised_error as sne
from make_golden import truth_solve_banded
ctx = mtg.Context(0)
N, D, K, r, B = 12, 1, 25, 5, 437
vals, mask, times = random_vertices_path_batch(N, D, K, B, seed0=3100 + K + D, max_derivative=4)
x = ctx.solve_linear_batch(N, r, vals, mask, times, status=True)
g = ctx.solve_linear_batch(N, r, vals, mask, times, general=True, status=True)
dg = np.array([sne(x["coeffs"][b:b + 1], g["coeffs"][b:b + 1], times[b:b + 1]) for b in range(B)])
order = np.argsort(dg)[::-1]
print("n>1e-8", int(np.sum(dg > 1e-8)), "median", np.median(dg))
for b in list(order[:4]) + list(order[200:202]):
    tr = truth_solve_banded(N, r, vals[b], mask[b], times[b])[None]
    sl = slice(b, b + 1)
    print(b, "dg %.2e" % dg[b], "x %.2e" % sne(x["coeffs"][sl], tr, times[sl]), "g %.2e" % sne(g["coeffs"][sl], tr, times[sl]),
          "tmin %.3g tmax %.3g" % (times[b].min(), times[b].max()), x["status"][b], g["status"][b], flush=True)
