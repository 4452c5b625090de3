#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.npz).

Inputs come from the restated reference generators (oracle/), the expected
outputs from a 60-digit mpmath evaluation of the reference algorithm itself
(lin_impl: Q(T) :574-589, A(T) :102-111, A^-1, H = A^-T Q A^-1, R = M^T H M
:298-326, R_pp d_p = -R_pf d_f :350-365, c = A^-1 M d :253-273, cost
0.5 sum c^T Q c :114-130).  At 60 digits every rounding difference between
the reference's FP64 path, the oracle and the GPU kernel is far below the
tolerances in tests/, so these are "truth" for all three.

This script is test infrastructure: it imports oracle/ (allowed for tests/).
Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import mpmath as mp
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
SNAP, JERK, ACCELERATION = 4, 3, 2
DPS = 60


def falling(n, i):
    if i < n:
        return 0
    out = 1
    for k in range(i - n + 1, i + 1):
        out *= k
    return out


def _system(N, r, vals, mask, times):
    """R = M^T H M of the reference (lin_impl:298-326) at 60 digits, with the fixed/free split and the
    per-segment A^-1 and Q."""
    mp.mp.dps = DPS
    h = N // 2
    V, nd, D = vals.shape
    K = V - 1
    msk = [int(m) & ((1 << h) - 1) for m in mask]
    fixed = [(v, k) for v in range(V) for k in range(h) if (msk[v] >> k) & 1]
    free = [(v, k) for v in range(V) for k in range(h) if not (msk[v] >> k) & 1]
    col = {c: i for i, c in enumerate(fixed + free)}
    n = len(fixed) + len(free)
    R = [[mp.mpf(0)] * n for _ in range(n)]
    Ainvs, Qs = [], []
    for i in range(K):
        T = mp.mpf(float(times[i]))
        A = mp.zeros(N, N)
        for k in range(h):
            A[k, k] = falling(k, k)
            for j in range(k, N):
                A[k + h, j] = falling(k, j) * T ** (j - k)
        Ai = mp.inverse(A)
        Q = mp.zeros(N, N)
        for a in range(r, N):
            for b in range(r, N):
                e = a + b - 2 * r + 1
                Q[a, b] = mp.mpf(2 * falling(r, a) * falling(r, b)) * T ** e / e
        H = Ai.T * Q * Ai
        Ainvs.append(Ai)
        Qs.append(Q)
        cols = [col[(i + (s >= h), s % h)] for s in range(N)]
        for a in range(N):
            for b in range(N):
                R[cols[a]][cols[b]] += H[a, b]
    return R, fixed, free, col, Ainvs, Qs


def truth_solve(N, r, vals, mask, times):
    """60-digit evaluation of the reference algorithm (see module doc)."""
    h = N // 2
    V, nd, D = vals.shape
    K = V - 1
    R, fixed, free, col, Ainvs, Qs = _system(N, r, vals, mask, times)
    nf, npf = len(fixed), len(free)
    df = [[mp.mpf(float(vals[v, k, d])) for (v, k) in fixed] for d in range(D)]
    dp = [[mp.mpf(0)] * npf for _ in range(D)]
    if npf:
        Rpp = mp.matrix([[R[nf + a][nf + b] for b in range(npf)] for a in range(npf)])
        for d in range(D):
            rhs = mp.matrix([-mp.fsum(R[nf + a][b] * df[d][b] for b in range(nf)) for a in range(npf)])
            sol = mp.lu_solve(Rpp, rhs)
            dp[d] = [sol[a] for a in range(npf)]
    coeffs = np.zeros((K, D, N))
    cost = mp.mpf(0)
    for i in range(K):
        cols = [col[(i + (s >= h), s % h)] for s in range(N)]
        for d in range(D):
            dall = df[d] + dp[d]
            dl = mp.matrix([dall[c] for c in cols])
            c = Ainvs[i] * dl
            coeffs[i, d] = [float(c[j]) for j in range(N)]
            cost += (c.T * Qs[i] * c)[0, 0]
    free_out = np.array([[float(x) for x in dp[d]] for d in range(D)]).reshape(D, npf)
    fixed_out = np.array([[float(x) for x in df[d]] for d in range(D)]).reshape(D, nf)
    return coeffs, float(cost / 2), free_out, fixed_out


def truth_solve_banded(N, r, vals, mask, times):
    """truth_solve's coefficients for long chains: the same 60-digit system (_system), R_pp solved by a
    banded LDL^T elimination (R_pp is block tridiagonal in the reference's (vertex, derivative) order,
    SPD, so no pivoting) instead of a dense LU -- O(n bw^2) instead of O(n^3) multiprecision operations
    (N = 10, K = 64: ~1 s instead of ~80 s).  Same digits: the tests use it where truth_solve is too
    slow (tests/test_oracle.py checks the two agree)."""
    h = N // 2
    V, nd, D = vals.shape
    K = V - 1
    R, fixed, free, col, Ainvs, Qs = _system(N, r, vals, mask, times)
    nf, npf = len(fixed), len(free)
    A = [[R[nf + a][nf + b] for b in range(npf)] for a in range(npf)]
    bw = 0
    for a in range(npf):
        for b in range(a + 1, npf):
            if A[a][b] != 0:
                bw = max(bw, b - a)
    for i in range(npf):  # in-place LDL^T (unit L below the diagonal, pivots on it)
        piv = A[i][i]
        for j in range(i + 1, min(npf, i + bw + 1)):
            f = A[i][j] / piv  # (the upper triangle is the updated one)
            if f == 0:
                continue
            for k in range(j, min(npf, i + bw + 1)):
                A[j][k] -= f * A[i][k]
            A[j][i] = f
    coeffs = np.zeros((K, D, N))
    for d in range(D):
        df = [mp.mpf(float(vals[v, k, d])) for (v, k) in fixed]
        x = [-mp.fsum(R[nf + a][b] * df[b] for b in range(nf)) for a in range(npf)]
        for i in range(npf):
            for j in range(i + 1, min(npf, i + bw + 1)):
                x[j] -= A[j][i] * x[i]
        for i in range(npf - 1, -1, -1):
            t = x[i] / A[i][i]
            for j in range(i + 1, min(npf, i + bw + 1)):
                t -= A[j][i] * x[j]
            x[i] = t
        dall = df + x
        for i in range(K):
            cols = [col[(i + (s >= h), s % h)] for s in range(N)]
            c = Ainvs[i] * mp.matrix([dall[c] for c in cols])
            coeffs[i, d] = [float(c[j]) for j in range(N)]
    return coeffs


def fp64_best_solve(N, r, vals, mask, times):
    """What a backward-stable FP64 solve reaches on this problem: R_pp and the right-hand side formed
    exactly (60 digits) and rounded once to FP64, equilibrated (symmetric diagonal scaling), solved
    by LU with partial pivoting (LAPACK via numpy), and mapped to coefficients with the correctly
    rounded A(T)^-1 in FP64, positions taken relative to each segment's start (else the mapping alone
    loses every digit of a millimetre segment far from the origin).  The arbiter for ill-conditioned problems (cond(R_pp) ~ 1e10 after
    equilibration): no FP64 solver can be expected to beat it by much."""
    h = N // 2
    V, nd, D = vals.shape
    K = V - 1
    R, fixed, free, col, Ainvs, Qs = _system(N, r, vals, mask, times)
    nf, npf = len(fixed), len(free)
    coeffs = np.zeros((K, D, N))
    Rf = np.array([[float(R[nf + a][nf + b]) for b in range(npf)] for a in range(npf)])
    sc = 1.0 / np.sqrt(np.abs(np.diag(Rf))) if npf else np.zeros(0)
    for d in range(D):
        df = [mp.mpf(float(vals[v, k, d])) for (v, k) in fixed]
        if npf:
            rhs = np.array([float(-mp.fsum(R[nf + a][b] * df[b] for b in range(nf))) for a in range(npf)])
            xp = np.linalg.solve(Rf * sc[:, None] * sc[None, :], rhs * sc) * sc
        else:
            xp = np.zeros(0)
        dall = np.concatenate([np.array([float(x) for x in df]), xp])
        for i in range(K):
            cols = [col[(i + (s >= h), s % h)] for s in range(N)]
            Ai = np.array([[float(Ainvs[i][a, b]) for b in range(N)] for a in range(N)])
            x = dall[cols].copy()
            p0 = x[0]
            if r >= 1:  # positions relative to the segment start (A^-1 maps a constant to c_0 only)
                x[0] -= p0
                x[h] -= p0
            coeffs[i, d] = Ai @ x
            if r >= 1:
                coeffs[i, d, 0] += p0
    return coeffs


def pack(problems):
    B = len(problems)
    V, nd, D = problems[0][0].shape
    K = V - 1
    vals = np.stack([p[0] for p in problems])
    mask = np.stack([p[1] for p in problems]).astype(np.uint32)
    times = np.stack([p[2] for p in problems])
    return vals, mask, times


def write_case(name, N, r, problems, note):
    t0 = time.time()
    vals, mask, times = pack(problems)
    B, V, nd, D = vals.shape
    K = V - 1
    coeffs, costs, frees, fixeds = [], [], [], []
    with ProcessPoolExecutor(max_workers=min(B, os.cpu_count() or 1)) as ex:
        res = list(ex.map(truth_solve, [N] * B, [r] * B, list(vals), list(mask), list(times)))
    for c, cost, fr, fx in res:
        coeffs.append(c)
        costs.append(cost)
        frees.append(fr)
        fixeds.append(fx)
    npf = max(f.shape[1] for f in frees)
    nfx = max(f.shape[1] for f in fixeds)
    free_pad = np.full((B, D, npf), np.nan)
    fixed_pad = np.full((B, D, nfx), np.nan)
    n_free = np.zeros(B, np.int32)
    n_fixed = np.zeros(B, np.int32)
    for b in range(B):
        free_pad[b, :, :frees[b].shape[1]] = frees[b]
        fixed_pad[b, :, :fixeds[b].shape[1]] = fixeds[b]
        n_free[b] = frees[b].shape[1]
        n_fixed[b] = fixeds[b].shape[1]
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, N=N, r=r, values=vals, mask=mask, times=times, coeffs=np.stack(coeffs),
                        cost=np.array(costs), free=free_pad, n_free=n_free, fixed=fixed_pad,
                        n_fixed=n_fixed, note=np.array(note))
    print("%-28s B=%-3d N=%-2d K=%-3d D=%d r=%d  %.1fs" % (name, B, N, K, D, r, time.time() - t0))


def cfg1(seeds):
    out = []
    for s in seeds:
        v, m = O.create_random_vertices(SNAP, 3, [-10, -20, -10], [10, 20, 10], s, nd=5)
        out.append((v, m, O.estimate_segment_times(v, 3.0, 5.0)))
    return out


def cfg2(seeds, K=10):
    out = []
    for s in seeds:
        v, m = O.create_random_vertices_path(3, K, 5.0, SNAP, s, nd=5)
        out.append((v, m, O.estimate_segment_times(v, 2.0, 2.0, 6.5)))
    return out


def cfg4(seeds, K=20):
    out = []
    for s in seeds:
        v, m = O.create_random_vertices(SNAP, K, [-10, -20, -10], [10, 20, 10], s, nd=6)
        out.append((v, m, O.estimate_segment_times(v, 3.0, 5.0)))
    return out


def mixed(seed, N, K, D, B):
    """Interior vertices with arbitrary per-vertex masks (position always set)."""
    rng = np.random.default_rng(seed)
    h = N // 2
    out = []
    for _ in range(B):
        v, m = O.create_random_vertices(h - 1 if h > 1 else 1, K, [-10] * D, [10] * D,
                                        int(rng.integers(1 << 30)), nd=max(h, 2))
        v = v[:, :h, :].copy() if v.shape[1] >= h else np.concatenate(
            [v, np.zeros((K + 1, h - v.shape[1], D))], axis=1)
        m = m & ((1 << h) - 1)
        for i in range(1, K):
            extra = int(rng.integers(0, 1 << h)) & ~1
            m[i] |= extra
            for k in range(1, h):
                if (extra >> k) & 1:
                    v[i, k, :] = rng.uniform(-2, 2, size=D)
        out.append((v, m.astype(np.uint32), rng.uniform(0.3, 4.0, size=K)))
    return out


def main(only=None):
    if only is not None:  # regenerate one case: python tests/golden/make_golden.py <name>
        global write_case
        _write = write_case

        def write_case(name, *a):
            if name == only:
                _write(name, *a)
    # 2_vertices_setup known answer (test/test_polynomial_optimization.cpp:700-744)
    v = np.zeros((2, 5, 1))
    v[1, 0, 0] = 5.0
    write_case("kat_2_vertices_setup", 10, 4, [(v, np.array([31, 31], np.uint32), np.array([5.0]))],
               "reference 2_vertices_setup, fully constrained, n_free=0")
    write_case("cfg1_n10_k3", 10, 4, cfg1([12345, 1, 2, 3, 4, 5, 6, 7]),
               "createRandomVertices(SNAP,3,[-10,-20,-10],[10,20,10],seed) + estimateSegmentTimes(3,5)")
    write_case("cfg2_n10_k10", 10, 4, cfg2(list(range(12))),
               "createRandomVerticesPath(3,10,5.0,SNAP,seed) + estimateSegmentTimes(2,2,6.5)")
    write_case("cfg4_n12_k20_jerk", 12, 3, cfg4(list(range(32))),
               "createRandomVertices(SNAP,20,[-10,-20,-10],[10,20,10],seed), r=JERK, times estimateSegmentTimes(3,5)")
    # ConstraintPacking shape: K=5, ends to JERK, D=3, N=10 default r=4
    cp = []
    for s in range(12345, 12345 + 6):
        v, m = O.create_random_vertices(JERK, 5, [-50] * 3, [50] * 3, s, nd=5)
        cp.append((v, m, O.estimate_segment_times(v, 3.0, 5.0)))
    write_case("constraint_packing_k5_jerk", 10, 4, cp, "ConstraintPacking shape (:777-836)")
    # 2_vertices_rand shape: K=1, ends to ACCELERATION (free jerk/snap at both ends)
    tv = []
    for s in range(12345, 12345 + 6):
        v, m = O.create_random_vertices(ACCELERATION, 1, [-50] * 3, [50] * 3, s, nd=5)
        tv.append((v, m, O.estimate_segment_times(v, 3.0, 5.0)))
    write_case("two_vertices_rand_acc", 10, 4, tv, "2_vertices_rand shape (:747-774)")
    write_case("mixed_n8_k6_d2_r2", 8, 2, mixed(7, 8, 6, 2, 6), "random interior masks, N=8, r=ACCELERATION")
    write_case("mixed_n12_k4_d4_r5", 12, 5, mixed(8, 12, 4, 4, 4), "random interior masks, N=12, r=5, D=4")
    write_case("mixed_n6_k5_d1_r1", 6, 1, mixed(9, 6, 5, 1, 4), "random interior masks, N=6, r=VELOCITY, D=1")
    write_case("n4_k8_d3_r0", 4, 0, mixed(10, 4, 8, 3, 3), "N=4, r=POSITION")
    write_case("cfg2_n10_k50", 10, 4, cfg2([100, 101], K=50), "bench generator, K=50")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
