"""IP kernel diagnosis: the default kernel vs MTG_FLAG_IP_KERNEL on config-2 problems (library from
MTG_LIBRARY), scale-normalised difference and event-timed kernel times."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402

res = {"lib": os.environ.get("MTG_LIBRARY", "default")}
for B in (10000, 125000):
    vals, mask, times = mtg.random_vertices_path_batch(10, 3, 10, B, seed0=0)
    dev = torch.device("cuda", 0)
    v, m, t = (torch.from_numpy(x).to(dev) for x in (vals, mask, times))
    ctx = mtg.Context(0)
    outs = {}
    for name, kw in (("default", {}), ("ip", {"ip": True})):
        o = torch.full((B, 10, 3, 10), float("nan"), dtype=torch.float64, device=dev)
        call = ctx.solve_call(10, 4, v, m, t, o, **kw)
        for _ in range(20):
            call()
        ctx.enable_timing(50)
        for _ in range(50):
            call()
        ms = float(np.median(ctx.kernel_times_ms(50)))
        outs[name] = o.cpu().numpy()
        res["%s_%d_ms" % (name, B)] = ms
    a, b = outs["default"], outs["ip"]
    tp = np.power(times[..., None], np.arange(10))[:, :, None, :]
    sc = np.max(np.abs(a) * tp, axis=-1)
    res["maxdiff_%d" % B] = float(np.nanmax(np.max(np.abs(a - b) * tp, axis=-1) / sc))
    res["ip_nan_%d" % B] = int(np.isnan(b).sum())
    res["bitequal_%d" % B] = bool(np.array_equal(a, b))
print(json.dumps(res))
