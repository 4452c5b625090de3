#!/usr/bin/env python3
"""Fixed cost of a timed region of K solve launches (bench.py's bracket: synchronize, K launches,
synchronize): wall time vs K with the closing wait done by torch.cuda.synchronize() alone, or by
polling an event recorded after the last launch and then synchronize(); median over 50 regions.

Run on the GPU box: python scripts/sync_overhead.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, N, D, K, r = 10000, 10, 3, 10, 4
    vals, mask, times = mtg.random_vertices_path_batch(N, D, K, B, seed0=0)
    v, m, t = (torch.from_numpy(x).to(dev) for x in (vals, mask, times))
    out = torch.empty((B, K, D, N), dtype=torch.float64, device=dev)
    ctx = mtg.Context(0)
    step = ctx.solve_call(N, r, v, m, t, out)
    stream = torch.cuda.current_stream(dev)
    for _ in range(3000):
        step()
    torch.cuda.synchronize(dev)
    res = {}
    for mode in ("sync", "poll"):
        for k in (1, 5, 20, 100):
            xs = []
            for _ in range(50):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(k):
                    step()
                if mode == "poll":
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    while not ev.query():
                        pass
                torch.cuda.synchronize(dev)
                xs.append(time.perf_counter() - t0)
            res["%s_%d_us" % (mode, k)] = float(np.median(xs) * 1e6)
        # fixed cost = intercept of the wall time vs k (least squares over the four k)
        ks = np.array([1, 5, 20, 100], dtype=float)
        ys = np.array([res["%s_%d_us" % (mode, k)] for k in (1, 5, 20, 100)])
        slope, icpt = np.polyfit(ks, ys, 1)
        res["%s_per_launch_us" % mode] = float(slope)
        res["%s_fixed_us" % mode] = float(icpt)
    # one launch's host time (enqueue only)
    torch.cuda.synchronize(dev)
    hs = []
    for _ in range(200):
        t0 = time.perf_counter()
        step()
        hs.append(time.perf_counter() - t0)
        torch.cuda.synchronize(dev)
    res["host_enqueue_us_median"] = float(np.median(hs) * 1e6)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
