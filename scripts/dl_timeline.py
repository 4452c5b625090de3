#!/usr/bin/env python3
"""Per-wave phase times of the dimension-lane kernel (debug build: cmake -DMTG_PHASE_TIMING=ON ->
lib_timing/): s_memrealtime stamps (100 MHz) at wave start, after the inputs landed, after the forward
sweep, after the backward sweep and after the wave's stores drained, with the wave's SIMD / CU / XCD.
Shows where a launch's time goes when all its waves run in one round (config 2, B = 1e4).

Run: MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so \\
     B=10000 python scripts/dl_timeline.py
"""
import collections
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (share torch's HIP runtime)
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402

B = int(os.environ.get("B", "10000"))
N, K, D = int(os.environ.get("N", "10")), int(os.environ.get("K", "10")), 3
r = 4 if N == 10 else 3
if os.environ.get("PATTERN") == "accel-ends":  # (the general-mask pass: ends fixed to ACCELERATION)
    vals, mask, times = mtg.random_vertices_batch(N, D, K, B, [-50.0] * 3, [50.0] * 3, seed0=0, max_derivative=2,
                                                  v_max=3.0, a_max=5.0)
elif N == 12:
    vals, mask, times = mtg.random_vertices_batch(N, D, K, B, [-10.0, -20.0, -10.0], [10.0, 20.0, 10.0], seed0=0,
                                                  max_derivative=4, v_max=3.0, a_max=5.0)
else:
    vals, mask, times = mtg.random_vertices_path_batch(N, D, K, B, seed0=0)
ctx = mtg.Context(0)
dev = torch.device("cuda", 0)
v_d, m_d, t_d = (torch.from_numpy(a).to(dev) for a in (vals, mask, times))
c_d = torch.empty((B, K, D, N), dtype=torch.float64, device=dev)
H = N // 2
fr_d = torch.zeros((B, D * (K + 1) * H), dtype=torch.float64, device=dev)
assert mtg._native.solve_kernel(N, D, K, r, B=B) == "solve_dl_kernel"
step = ctx.solve_call(N, r, v_d, m_d, t_d, c_d, free=fr_d)
for _ in range(20):
    step()
torch.cuda.synchronize()
f = fr_d.cpu().numpy()
tpw = 64 // (2 * D)
w = f[::tpw]
st = w[:, :5]
t0 = st[:, 0].min()
rel = (st - t0) * 10.0 / 1e3  # us
hw = w[:, 5].astype(np.int64)
xcc = w[:, 6].astype(np.int64)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
key = list(zip(xcc, se, cu, simd))
per_simd = collections.Counter(key)
ph = np.diff(st, axis=1) * 10.0 / 1e3
names = ["loads", "forward", "backward", "drain"]
res = {"B": B, "N": N, "K": K, "waves": int(len(w)), "span_us": float(rel[:, 4].max()),
       "start_us": {"p50": float(np.percentile(rel[:, 0], 50)), "max": float(rel[:, 0].max())},
       "phase_us_mean": {n: float(ph[:, i].mean()) for i, n in enumerate(names)},
       "phase_us_p90": {n: float(np.percentile(ph[:, i], 90)) for i, n in enumerate(names)},
       "end_us": {"p10": float(np.percentile(rel[:, 4], 10)), "p50": float(np.percentile(rel[:, 4], 50)),
                  "max": float(rel[:, 4].max())},
       "simds_used": len(per_simd),
       "simds_by_wave_count": {int(k): int(v) for k, v in sorted(collections.Counter(per_simd.values()).items())},
       "waves_per_xcd": {int(k): int(v) for k, v in sorted(collections.Counter(xcc).items())}}
# per XCD, relative to its own first wave (the XCDs' clocks may be offset)
res["per_xcd"] = {}
for x in sorted(set(xcc.tolist())):
    sel = xcc == x
    s0 = st[sel, 0].min()
    res["per_xcd"][int(x)] = {"start_p50_us": float(np.percentile(st[sel, 0] - s0, 50) / 100),
                              "start_max_us": float((st[sel, 0] - s0).max() / 100),
                              "span_us": float((st[sel, 4] - s0).max() / 100)}
print(json.dumps(res))
