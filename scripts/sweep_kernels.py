#!/usr/bin/env python3
"""Kernel time (HIP events in the dispatch packet, mean of 64 launches after 64 warmups) of the
config-2 solve vs batch size, for the kernels named in KERNELS (column, dl, default, general), in one process.

Run on the GPU box: python scripts/sweep_kernels.py [B ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402

Bs = [int(x) for x in sys.argv[1:]] or [1024, 8192, 8224, 9216, 10000, 12288, 16384, 24576, 32768, 65536, 131072]
vals, mask, times = mtg.random_vertices_path_batch(10, 3, 10, max(Bs), seed0=0)
dev = torch.device("cuda", 0)
v_d, m_d, t_d = (torch.from_numpy(x).to(dev) for x in (vals, mask, times))
out = torch.empty((max(Bs), 10, 3, 10), dtype=torch.float64, device=dev)
ctx = mtg.Context(0)
for B in Bs:
    row = {"B": B}
    kinds = (("column", {"column": True}), ("dl", {"dl": True}), ("default", {}), ("general", {"general": True}))
    for name, kw in [k for k in kinds if k[0] in os.environ.get("KERNELS", "column,dl").split(",")]:
        step = ctx.solve_call(10, 4, v_d[:B], m_d[:B], t_d[:B], out[:B], **kw)
        ctx.enable_timing(0)
        for _ in range(64):
            step()
        ctx.enable_timing(64)
        for _ in range(64):
            step()
        ms = ctx.kernel_times_ms(64)
        row[name] = round(float(np.mean(ms)) * 1e3, 2)
    row["lib"] = os.environ.get("MTG_LIBRARY", "default")
    print(row, flush=True)
