#!/usr/bin/env python3
"""Bitwise fixture of the host solve (mtg_host_solve_linear_batch) taken from the full-layout sweep
it had before commit f6a01fe (round 4), which restricted the forward and backward sweeps to each
vertex's free derivatives and was claimed bit-identical (the pinned rows and columns only added
exact zeros).  This script builds that earlier mtg_host_solve.cpp from git (commit 46c85dc) with the
library's own host flags (-O3 -ffp-contract=off) and records its outputs on mask patterns that
exercise the claim: fully pinned and fully free vertices, free end derivatives, every pin subset,
several N / D / r and odd and even K.  tests/test_host_solver.py::test_host_solve_bitwise_fixture
compares the current host solve with it bit for bit.  Test infrastructure; run from the repo root:
    python tests/golden/make_host_fixture.py
"""
import ctypes
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
COMMIT = "46c85dc"
CASES = [(10, 3, 10, 4), (10, 3, 7, 4), (12, 3, 20, 3), (8, 2, 5, 2), (6, 1, 4, 1), (12, 4, 3, 5), (4, 3, 6, 0)]


def build_old(tmp):
    src = os.path.join(tmp, "mtg_host_solve_old.cpp")
    with open(src, "w") as f:
        f.write(subprocess.run(["git", "-C", ROOT, "show", COMMIT + ":mav_trajectory_generation_cmake_amd/csrc/mtg_host_solve.cpp"],
                               check=True, capture_output=True, text=True).stdout)
    so = os.path.join(tmp, "libhs_old.so")
    csrc = os.path.join(ROOT, "mav_trajectory_generation_cmake_amd", "csrc")
    subprocess.run(["g++", "-O3", "-DNDEBUG", "-std=gnu++17", "-fPIC", "-ffp-contract=off", "-shared", "-I",
                    os.path.join(ROOT, "include"), "-I", csrc, src, "-o", so, "-pthread"], check=True)
    return so


def problems(N, D, K, seed):
    sys.path.insert(0, ROOT)
    import mav_trajectory_generation_cmake_amd as mtg
    h = N // 2
    B = 18
    vals, mask, times = mtg.random_vertices_path_batch(N, D, K, B, seed0=seed, max_derivative=min(4, h - 1))
    rng = np.random.default_rng(seed)
    vals, mask = vals.copy(), mask.copy()
    vals[:, :, 1:, :] = rng.normal(size=vals[:, :, 1:, :].shape)
    full = (1 << h) - 1
    for b in range(B):
        kind = b % 6
        if kind == 1:      # random pins, positions fixed
            mask[b] = (rng.integers(0, 1 << h, size=K + 1) | 1).astype(np.uint8)
        elif kind == 2:    # a fully pinned interior vertex and a fully free one
            mask[b, K // 2] = full
            if K >= 3:
                mask[b, 1] = 0
        elif kind == 3:    # free end derivatives above the position
            mask[b, 0] = mask[b, -1] = 1
        elif kind == 4:    # every derivative pinned everywhere except one interior vertex
            mask[b, :] = full
            if K >= 2:
                mask[b, K // 2] = 1
        elif kind == 5:    # random pins including free positions (ends fixed)
            mask[b] = rng.integers(0, 1 << h, size=K + 1).astype(np.uint8)
            mask[b, 0] = mask[b, -1] = full
    return vals, mask, times


def run(lib, N, D, K, r, vals, mask, times):
    B = vals.shape[0]
    V, h = K + 1, N // 2
    c = np.empty((B, K, D, N))
    fr = np.zeros((B, D, V * h))
    nf = np.empty((B,), np.int32)
    co = np.empty((B,))
    st = np.empty((B,), np.int32)
    p = lambda a: ctypes.c_void_p(a.ctypes.data)
    rc = lib.mtg_host_solve_linear_batch(N, D, K, r, ctypes.c_int64(B), p(vals), p(mask), p(times), p(c), p(fr), p(nf),
                                         p(co), p(st), 1)
    assert rc == 0, rc
    return c, fr, nf, co, st


def main():
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        lib = ctypes.CDLL(build_old(tmp))
        for i, (N, D, K, r) in enumerate(CASES):
            vals, mask, times = problems(N, D, K, 100 + i)
            c, fr, nf, co, st = run(lib, N, D, K, r, vals, mask, times)
            key = "n%d_d%d_k%d_r%d" % (N, D, K, r)
            for name, a in (("values", vals), ("mask", mask), ("times", times), ("coeffs", c), ("free", fr),
                            ("n_free", nf), ("cost", co), ("status", st)):
                out[key + "__" + name] = a
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "host_solve_bitwise.npz"), commit=COMMIT, **out)
    print("wrote tests/golden/host_solve_bitwise.npz (%d cases, host solve of %s)" % (len(CASES), COMMIT))


if __name__ == "__main__":
    main()
