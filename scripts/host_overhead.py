#!/usr/bin/env python3
"""Host-side cost of one bench step (ctypes + C ABI + launch), against the GPU time per step:
submits 2000 asynchronous device-pointer solves and times the submission loop alone, then the
drain.  If the submission rate is below the kernel rate the bench's wall clock is host-bound."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402

B = int(os.environ.get("B", "10000"))
dev = torch.device("cuda", 0)
vals, mask, times = mtg.random_vertices_path_batch(10, 3, 10, B, seed0=0)
ctx = mtg.Context(0)
v_d, m_d, t_d = (torch.from_numpy(x).to(dev) for x in (vals, mask, times))
c_d = torch.empty((B, 10, 3, 10), dtype=torch.float64, device=dev)
step = ctx.solve_call(10, 4, v_d, m_d, t_d, c_d)
timing = os.environ.get("TIMING", "1") == "1"
ctx.enable_timing(2000 if timing else 0)
for _ in range(20):
    step()
torch.cuda.synchronize()
n = 2000
t0 = time.perf_counter()
for _ in range(n):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
k = float(np.mean(ctx.kernel_times_ms(n))) if timing else float("nan")
print("B=%d submit %.2f us/step, wall %.2f us/step, kernel %.2f us" % (B, (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6,
                                                                     k * 1e3))
