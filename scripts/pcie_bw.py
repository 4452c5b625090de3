"""Host <-> device copy rates on the box (torch, one GPU): pinned vs pageable, each direction alone
and H2D + D2H concurrently on two streams.  Informs the chunk pipeline of run_solve_pipelined."""
import json
import time

import torch


def rate(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


out = {}
for mb in (8, 32, 128, 512):
    n = mb << 20
    hp = torch.empty(n, dtype=torch.uint8).pin_memory()
    hq = torch.empty(n, dtype=torch.uint8)
    hq.fill_(1)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    hp2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    r = {}
    r["h2d_pinned"] = rate(lambda: d.copy_(hp, non_blocking=True), n)
    r["h2d_pageable"] = rate(lambda: d.copy_(hq), n)
    r["d2h_pinned"] = rate(lambda: hp.copy_(d, non_blocking=True), n)
    r["d2h_pageable"] = rate(lambda: hq.copy_(d), n)

    def both():
        with torch.cuda.stream(s1):
            d.copy_(hp, non_blocking=True)
        with torch.cuda.stream(s2):
            hp2.copy_(d2, non_blocking=True)
    r["duplex_pinned_total"] = rate(both, 2 * n)
    out[mb] = {k: round(v, 1) for k, v in r.items()}
    print(mb, "MB", out[mb], flush=True)
print(json.dumps(out))
