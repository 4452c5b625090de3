# Diagnose the accuracy of trajectory 8030 (bench generator seed 8030): GPU free values vs
# 60-digit truth, and recovery of coefficients from them on the host.
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests", "golden"))
import numpy as np
import mav_trajectory_generation_cmake_amd as m
from _util import scale_normalised_error
from make_golden import truth_solve
v, mk, t = m.random_vertices_path_batch(10, 3, 10, 1, seed0=8030)
ctx = m.Context(0)
out = ctx.solve_linear_batch(10, 4, v, mk, t, free=True, n_free=True, cost=True)
tr, cost, free_tr, _ = truth_solve(10, 4, v[0], mk[0], t[0])
nf = int(out["n_free"][0])
fr = out["free"][0][:, :nf]
print("coeff err", scale_normalised_error(out["coeffs"], tr[None], t))
print("free rel err per dim", np.max(np.abs(fr - free_tr), axis=1) / np.max(np.abs(free_tr), axis=1))
print("free abs err by entry (dim0)", np.abs(fr - free_tr)[0])
print("free truth (dim0)", free_tr[0])
print("cost", out["cost"][0], cost)
np.savez("gpurun_out/debug_8030.npz", coeffs=out["coeffs"], free=fr, truth=tr, free_truth=free_tr)
