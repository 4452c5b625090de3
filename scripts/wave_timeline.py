#!/usr/bin/env python3
"""Per-wave start/end times and placement of the register column kernel (debug build:
cmake -DMTG_PHASE_TIMING=ON).  Shows whether a launch is bound by the slowest SIMD's resident waves
or by waves that start late (dispatch / residency), and how evenly waves spread over XCDs and SIMDs.

Run: MTG_LIBRARY=mav_trajectory_generation_cmake_amd/lib_timing/libmav_trajectory_generation.so \
     B=10000 python scripts/wave_timeline.py
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
vals, mask, times = mtg.random_vertices_path_batch(10, 3, 10, B, seed0=0)
ctx = mtg.Context(0)
dev = torch.device("cuda", 0)
v_d, m_d, t_d = (torch.from_numpy(a).to(dev) for a in (vals, mask, times))
c_d = torch.empty((B, 10, 3, 10), dtype=torch.float64, device=dev)
fr_d = torch.zeros((B, 3 * 11 * 5), dtype=torch.float64, device=dev)
step = ctx.solve_call(10, 4, v_d, m_d, t_d, c_d, free=fr_d)  # one device-pointer launch (as bench.py)
for _ in range(3):
    step()
torch.cuda.synchronize()
f = fr_d.cpu().numpy()
tpw = 4  # trajectories per wave (16 lanes each); the first of each wave carries the stamps
w = f[::tpw]
t0, t1 = w[:, 9], w[:, 10]  # s_memrealtime, 100 MHz
hw = w[:, 11].astype(np.int64)
xcc = w[:, 12].astype(np.int64)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
start = (t0 - t0.min()) * 10.0  # ns
end = (t1 - t0.min()) * 10.0
dur = end - start
key = list(zip(xcc, se, sh, cu, simd))
per_simd = collections.Counter(key)
occ = collections.Counter(per_simd.values())
res = {
    "B": B, "waves": int(len(w)),
    "span_us": float(end.max() / 1e3),
    "start_us": {"p50": float(np.percentile(start, 50) / 1e3), "p90": float(np.percentile(start, 90) / 1e3),
                 "max": float(start.max() / 1e3)},
    "dur_us": {"min": float(dur.min() / 1e3), "p50": float(np.percentile(dur, 50) / 1e3),
               "p90": float(np.percentile(dur, 90) / 1e3), "max": float(dur.max() / 1e3)},
    "waves_per_xcd": {int(k): int(v) for k, v in sorted(collections.Counter(xcc).items())},
    "simds_used": len(per_simd),
    "simds_by_wave_count": {int(k): int(v) for k, v in sorted(occ.items())},
    "phase_cycles_mean": {n: float(f[:, i].mean()) for i, n in enumerate(["staging", "forward", "backward", "epilogue"])},
    "forward_sub_cycles_mean": {n: float(w[:, 4 + i].mean()) for i, n in enumerate(["products", "exchange", "factor_solve"])},
    "epilogue_sub_cycles_mean": {"a1_load": float(w[:, 7].mean()), "stores": float(w[:, 8].mean())},
}
# duration by the number of waves sharing the SIMD
by = collections.defaultdict(list)
for k, d in zip(key, dur):
    by[per_simd[k]].append(d)
res["dur_us_by_simd_waves"] = {int(k): float(np.mean(v) / 1e3) for k, v in sorted(by.items())}
# late starters: waves that start after the first finished
slow = dur >= np.percentile(dur, 90)
res["slowest_decile_phase_cycles"] = {n: float(w[slow, i].mean()) for i, n in enumerate(["staging", "forward", "backward", "epilogue"])}
# per XCD (each XCD's clock may be offset): start spread and span relative to its first wave
res["per_xcd"] = {}
for x in sorted(set(xcc.tolist())):
    sel = xcc == x
    s0 = t0[sel].min()
    res["per_xcd"][int(x)] = {"start_p50_us": float(np.percentile(t0[sel] - s0, 50) / 100),
                              "start_max_us": float((t0[sel] - s0).max() / 100),
                              "span_us": float((t1[sel] - s0).max() / 100)}
res["waves_starting_after_first_end_us"] = int((start > end.min()).sum())
print(json.dumps(res))
