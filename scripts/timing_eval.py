#!/usr/bin/env python3
"""Latency table mirroring the reference's only benchmark, src/polynomial_timing_evaluation.cpp:93-128:
createRandomVerticesPath(3, K, 5.0, SNAP, seed=1) + estimateSegmentTimes(2, 2, 6.5), then
PolynomialOptimization<10>(3) + setupFromVertices + solveLinear, for K in {2, 10, 50, 100}.

One JSON line per K:
  cpu_us          the oracle restatement on one core, per solve (the span the reference's timer covers)
  gpu_call_us     one trajectory per mtg_solve_linear_batch call with host arrays (staging H2D, kernel,
                  D2H, synchronize): the drop-in PolynomialOptimization::solveLinear latency
  gpu_batch_us    the same problem x 10000 in one device-resident call, per trajectory
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402
from oracle import pyoracle  # noqa: E402  (the CPU column only)

N, r, D = 10, 4, 3
lib = pyoracle.build(build_dir="_build_bench", arch=os.environ.get("MTG_ORACLE_ARCH", "native"))
pyoracle._LIB = None
pyoracle.lib(lib)
ctx = mtg.Context(0)
dev = torch.device("cuda", 0)


def rate(fn, max_n=1000, budget_s=2.0, min_n=3):
    n, t0 = 0, time.perf_counter()
    while n < max_n and (n < min_n or time.perf_counter() - t0 < budget_s):
        fn()
        n += 1
    return (time.perf_counter() - t0) / n * 1e6, n


for K in (2, 10, 50, 100):
    vals, mask, times = mtg.random_vertices_path_batch(N, D, K, 1, seed0=1)
    m32 = mask.astype(np.uint32)
    cpu_us, cpu_n = rate(lambda: pyoracle.solve_linear_batch(N, r, vals, m32, times, threads=1))
    for _ in range(5):
        ctx.solve_linear_batch(N, r, vals, mask, times)
    call_us, call_n = rate(lambda: ctx.solve_linear_batch(N, r, vals, mask, times))
    Bb = 10000
    v_d = torch.from_numpy(np.repeat(vals, Bb, axis=0)).to(dev)
    m_d = torch.from_numpy(np.repeat(mask, Bb, axis=0)).to(dev)
    t_d = torch.from_numpy(np.repeat(times, Bb, axis=0)).to(dev)
    c_d = torch.empty((Bb, K, D, N), dtype=torch.float64, device=dev)
    step = ctx.solve_call(N, r, v_d, m_d, t_d, c_d)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        step()
    torch.cuda.synchronize()
    batch_us = (time.perf_counter() - t0) / 50 / Bb * 1e6
    ctx.reset_stream()
    print(json.dumps({"K": K, "cpu_us": round(cpu_us, 2), "cpu_solves": cpu_n, "cpu_threads": 1,
                      "gpu_call_us": round(call_us, 2), "gpu_calls": call_n,
                      "gpu_batch_us_per_traj": round(batch_us, 5)}), flush=True)
