#!/usr/bin/env python3
"""Trajectory::computeMinMaxMagnitude throughput (include/mtg.h
mtg_min_max_magnitude_batch): config-2 trajectories solved on the GPU, then the minimum and maximum
of |p^(k)| over each whole trajectory (k = 0 position, and 2 acceleration), device-resident.
Prints trajectories/s and the kernel time (HIP events in the dispatch packet).

Run on the GPU box: python scripts/bench_extrema.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402
from mav_trajectory_generation_cmake_amd import _native as nat  # noqa: E402
from mav_trajectory_generation_cmake_amd.solver import EXTREMUM_DTYPE, _addr  # noqa: E402

B = int(os.environ.get("B", "10000"))
steps = int(os.environ.get("STEPS", "20"))
N, D, K, r = 10, 3, 10, 4
vals, mask, times = mtg.random_vertices_path_batch(N, D, K, B, seed0=0)
ctx = mtg.Context(0)
coeffs = ctx.solve_linear_batch(N, r, vals, mask, times)["coeffs"]
dev = torch.device("cuda", 0)
c_d = torch.from_numpy(coeffs).to(dev)
t_d = torch.from_numpy(times).to(dev)
nbytes = EXTREMUM_DTYPE.itemsize * B
mn_d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
mx_d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
lib = ctx._lib
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
F = nat.MTG_FLAG_DEVICE_PTRS | nat.MTG_FLAG_ASYNC
res = {"B": B, "workload": "config2 trajectories (K=10, N=10, D=3), whole-trajectory min/max of |p^(k)|"}
for deriv in (0, 2):
    def run():
        nat.check(lib.mtg_min_max_magnitude_batch(ctx.handle, N, D, K, B, _addr(c_d), _addr(t_d), deriv, 0,
                                                  _addr(mn_d), _addr(mx_d), F), ctx.handle)
    ctx.enable_timing(0)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    ctx.enable_timing(steps)
    for _ in range(steps):
        run()
    kms = float(np.mean(ctx.kernel_times_ms(steps)))
    # spot check against the host-array path (same kernel) and the oracle's candidates (tests do the full check)
    mn_h, mx_h = ctx.min_max_magnitude_batch(coeffs[:64], times[:64], deriv)
    got_mx = np.frombuffer(mx_d.cpu().numpy().tobytes(), dtype=EXTREMUM_DTYPE)[:64]
    assert np.array_equal(got_mx["value"], mx_h["value"])
    res["derivative_%d" % deriv] = {"kernel_ms": kms, "trajectories_per_s": B / (kms * 1e-3),
                                    "segments_per_s": B * K / (kms * 1e-3)}
print(json.dumps(res))
