#!/usr/bin/env python3
"""end_to_end diagnosis: host-array solves through the C ABI from pageable arrays and
from pinned arrays allocated three ways -- torch pin_memory() from wherever the process runs, pinned
memory first-touched by a thread bound to the GPU's NUMA node, and the torch buffers called from a
thread bound to that node -- interleaved call by call, median and 10/90 percentiles.  Reports the
NUMA node of each buffer's pages (move_pages) and of the GPU.

Run on the GPU box: python scripts/e2e_diag.py [B ...]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mav_trajectory_generation_cmake_amd as mtg  # noqa: E402

libc = ctypes.CDLL(None, use_errno=True)
PAGE = os.sysconf("SC_PAGE_SIZE")


def page_nodes(arr, samples=64):
    """NUMA nodes of a sample of the array's pages (move_pages with nodes = NULL reports them)."""
    base = arr.ctypes.data
    n = max(1, arr.nbytes // PAGE)
    idx = np.unique(np.linspace(0, n - 1, min(samples, n)).astype(np.int64))
    pages = (ctypes.c_void_p * len(idx))(*[(base // PAGE + int(i)) * PAGE for i in idx])
    status = (ctypes.c_int * len(idx))()
    rc = libc.syscall(279, 0, len(idx), pages, None, status, 0)  # SYS_move_pages (x86_64)
    if rc != 0:
        return "move_pages failed (errno %d)" % ctypes.get_errno()
    vals, counts = np.unique(np.array(status[:]), return_counts=True)
    return {int(v): int(c) for v, c in zip(vals, counts)}


def gpu_node():
    p = torch.cuda.get_device_properties(0)
    path = "/sys/bus/pci/devices/%04x:%02x:%02x.0/numa_node" % (getattr(p, "pci_domain_id", 0), p.pci_bus_id,
                                                                 p.pci_device_id)
    try:
        return int(open(path).read()), path
    except OSError as e:
        return -1, str(e)


def node_cpus(node):
    def parse(s):
        out = set()
        for part in s.strip().split(","):
            if not part:
                continue
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
        return out
    try:
        cpus = parse(open("/sys/devices/system/node/node%d/cpulist" % node).read())
    except OSError:
        return set()
    return cpus & os.sched_getaffinity(0)


def main():
    Bs = [int(x) for x in sys.argv[1:]] or [10000, 125000]
    node, npath = gpu_node()
    local = node_cpus(node) if node >= 0 else set()
    allcpus = os.sched_getaffinity(0)
    res = {"gpu_numa_node": node, "numa_path": npath, "affinity_cpus": len(allcpus), "gpu_node_cpus": len(local),
           "nodes": sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node"))}
    ctx = mtg.Context(0)
    N, D, K, r = 10, 3, 10, 4
    for B in Bs:
        vals, mask, times = mtg.random_vertices_path_batch(N, D, K, B, seed0=0)
        page_out = np.empty((B, K, D, N))
        torch_in = [torch.from_numpy(x).pin_memory().numpy() for x in (vals, mask, times)]
        torch_out = torch.empty((B, K, D, N), dtype=torch.float64).pin_memory().numpy()
        modes = [("pageable", (vals, mask, times), page_out, None),
                 ("pinned_torch", torch_in, torch_out, None)]
        if local:
            # pinned memory allocated (and so first touched) by this thread while bound to the GPU's node
            os.sched_setaffinity(0, local)
            loc_in = [torch.from_numpy(x.copy()).pin_memory().numpy() for x in (vals, mask, times)]
            loc_out = torch.empty((B, K, D, N), dtype=torch.float64).pin_memory().numpy()
            os.sched_setaffinity(0, allcpus)
            modes.append(("pinned_local", loc_in, loc_out, None))
            modes.append(("pinned_torch_caller_local", torch_in, torch_out, local))
            modes.append(("pageable_caller_local", (vals, mask, times), page_out, local))
        row = {"B": B, "buffers": {m[0]: {"in": page_nodes(m[1][0]), "out": page_nodes(m[2])} for m in modes}}
        for _ in range(3):
            for _, (v, m, t), o, cpus in modes:
                ctx.solve_linear_batch(N, r, v, m, t, coeffs=o)
        secs = {m[0]: [] for m in modes}
        for _ in range(30):
            for name, (v, m, t), o, cpus in modes:
                if cpus:
                    os.sched_setaffinity(0, cpus)
                t0 = time.perf_counter()
                ctx.solve_linear_batch(N, r, v, m, t, coeffs=o)
                secs[name].append(time.perf_counter() - t0)
                if cpus:
                    os.sched_setaffinity(0, allcpus)
        for name, x in secs.items():
            x = np.array(x) * 1e3
            row[name] = {"median_ms": float(np.median(x)), "p10_ms": float(np.percentile(x, 10)),
                         "p90_ms": float(np.percentile(x, 90)), "min_ms": float(x.min()), "max_ms": float(x.max())}
        res["B%d" % B] = row
        print(json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
