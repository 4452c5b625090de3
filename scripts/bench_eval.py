#!/usr/bin/env python3
"""evaluateRange throughput: config-2 trajectories solved on the GPU, then
Trajectory::evaluateRange(0, T_total, dt=0.01, POSITION) for the whole batch, device-resident.
Prints samples/s, output GB/s (D doubles per sample + the sample time) and the kernel times."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402
from mav_trajectory_generation_cmake_amd import _native as nat  # noqa: E402
from mav_trajectory_generation_cmake_amd.solver import _addr  # noqa: E402

B = int(os.environ.get("B", "10000"))
steps = int(os.environ.get("STEPS", "10"))
N, D, K, r, dt = 10, 3, 10, 4, 0.01
vals, mask, times = mtg.random_vertices_path_batch(N, D, K, B, seed0=0)
ctx = mtg.Context(0)
coeffs = ctx.solve_linear_batch(N, r, vals, mask, times)["coeffs"]
dev = torch.device("cuda", 0)
c_d = torch.from_numpy(coeffs).to(dev)
t_d = torch.from_numpy(times).to(dev)
cnt_d = torch.zeros(B, dtype=torch.int64, device=dev)
lib = ctx._lib
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
F = nat.MTG_FLAG_DEVICE_PTRS
t_end = 1e9
nat.check(lib.mtg_evaluate_range_batch(ctx.handle, N, D, K, B, None, _addr(t_d), 0.0, t_end, dt, 0, _addr(cnt_d),
                                       None, None, None, F), ctx.handle)
counts = cnt_d.cpu().numpy()
offs = np.zeros(B, dtype=np.int64)
offs[1:] = np.cumsum(counts)[:-1]
total = int(counts.sum())
o_d = torch.from_numpy(offs).to(dev)
out_d = torch.empty((total, D), dtype=torch.float64, device=dev)
st_d = torch.empty(total, dtype=torch.float64, device=dev)
ctx.enable_timing(steps)


def count():
    nat.check(lib.mtg_evaluate_range_batch(ctx.handle, N, D, K, B, None, _addr(t_d), 0.0, t_end, dt, 0,
                                           _addr(cnt_d), None, None, None, F | nat.MTG_FLAG_ASYNC), ctx.handle)


def run():
    nat.check(lib.mtg_evaluate_range_batch(ctx.handle, N, D, K, B, _addr(c_d), _addr(t_d), 0.0, t_end, dt, 0,
                                           _addr(cnt_d), _addr(o_d), _addr(out_d), _addr(st_d),
                                           F | nat.MTG_FLAG_ASYNC), ctx.handle)


for _ in range(2):
    count()
    run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    count()
torch.cuda.synchronize()
t_count = (time.perf_counter() - t0) / steps
t0 = time.perf_counter()
for _ in range(steps):
    run()
torch.cuda.synchronize()
t_run = (time.perf_counter() - t0) / steps
kms = float(np.mean(ctx.kernel_times_ms(steps)))
# spot-check against the oracle's evaluateRange on a few trajectories (bit-exact)
from oracle import pyoracle as O  # noqa: E402
out = out_d.cpu().numpy()
st = st_d.cpu().numpy()
for b in (0, B // 2, B - 1):
    ro, rst, n = O.evaluate_range(coeffs[b], times[b], 0.0, t_end, dt, 0, max_samples=int(counts[b]) + 10)
    assert n == counts[b] and np.array_equal(out[offs[b]:offs[b] + n], ro) and np.array_equal(st[offs[b]:offs[b] + n], rst)
bytes_out = total * (D + 1) * 8
print(json.dumps({"B": B, "samples": total, "samples_per_traj": total / B, "count_ms": t_count * 1e3,
                  "eval_ms_wall": t_run * 1e3, "eval_kernel_ms": kms, "samples_per_s": total / (kms * 1e-3),
                  "out_GBps": bytes_out / (kms * 1e-3) / 1e9, "frac_hbm": bytes_out / (kms * 1e-3) / 8e12}))
