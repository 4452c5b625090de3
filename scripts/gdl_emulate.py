#!/usr/bin/env python3
"""Numpy emulation of the dimension-lane kernel's GENERAL-mask mode (mtg_solve_dl.inc, "GDL"):
any per-vertex mask that fixes the position at every vertex, the other derivatives fixed or free.
The twisted scaled-basis block LDL^T of DESIGN.md 3.2c with runtime pinning: pinned rows / columns
of S'_J are zeroed with 1 / pivot 0, pinned entries of z'_J carry the fixed values, and the fixed
values' couplings (own vertex TL~ + rho^e BR~, next vertex BL~^T T^(b+1)) move to the right-hand
side.  Checked against the oracle (the reference algorithm, lin_impl:298-369) on random masks.
Usage: python scripts/gdl_emulate.py [N K R trials]   (test infrastructure; not product code)"""
import os
import sys
from fractions import Fraction

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mav_trajectory_generation_cmake_amd", "csrc"))
import gen_tables  # noqa: E402


def htilde(N, R):
    return np.array([[float(x) for x in row] for row in gen_tables.tables()[("HTILDE", N, R)]])


def a1inv(N):
    return np.array([[float(x) for x in row] for row in gen_tables.tables()[("A1INV", N)]])


def factor_pinned(S, pin):
    """LDL^T of S (F x F) with pinned rows / columns: L zero there, dinv 0."""
    F = len(S)
    S = S.copy()
    for a in range(F):
        for b in range(F):
            if pin[a] or pin[b]:
                S[a, b] = 0.0
    L = np.eye(F)
    dg = np.zeros(F)
    dinv = np.zeros(F)
    for j in range(F):
        dj = S[j, j] - sum(L[j, k] ** 2 * dg[k] for k in range(j))
        if not pin[j]:
            dg[j] = dj
            dinv[j] = 1.0 / dj
        for i in range(j + 1, F):
            t = S[i, j] - sum(L[i, k] * L[j, k] * dg[k] for k in range(j))
            L[i, j] = 0.0 if pin[j] else t * dinv[j]
    return L, dinv


def solve(L, dinv, y):
    y = y.copy()
    F = len(y)
    for i in range(F):
        y[i] -= L[i, :i] @ y[:i]
    for i in range(F - 1, -1, -1):
        y[i] = y[i] * dinv[i] - L[i + 1:, i] @ y[i + 1:]
    return y


def chain_view(vals, mask, times, ch):
    """Chain A: the trajectory as given; chain B: time-reversed (odd derivatives negated)."""
    if ch == 0:
        return vals, mask, times
    v = vals[::-1].copy()
    sgn = np.array([(-1.0) ** k for k in range(vals.shape[1])])
    return v * sgn[:, None], mask[::-1].copy(), times[::-1].copy()


def emulate(N, R, vals, mask, times):
    """One trajectory, vals [V][H][D], mask [V], times [K]: coefficients [K][D][N]."""
    H, F = N // 2, N // 2 - 1
    K = len(times)
    KC = K // 2
    assert K % 2 == 0
    Ht = htilde(N, R)
    TL = Ht[1:H, 1:H]
    BR = Ht[H + 1:, H + 1:]
    BL = Ht[H + 1:, 1:H]       # BL[a][k]
    hp = Ht[H + 1:, H]
    hn = Ht[1:H, H]
    D = vals.shape[2]
    out = {}
    halves = {}
    st = {}
    for ch in (0, 1):
        v, m, T = chain_view(vals, mask, times, ch)
        pin = [[bool((m[j] >> (a + 1)) & 1) for a in range(F)] for j in range(K + 1)]
        assert all(m[j] & 1 for j in range(K + 1))
        f = v[:, 1:H, :]        # fixed values (chain coordinates), [V][F][D]
        P = v[:, 0, :]
        Ls, Ds, Zs = [], [], []
        # vertex 0: S' = TL~, rhs' = -(hn dpn + TL~ Yf_0 + BL~^T T_0^(b+1) f_1)
        t0 = T[0]
        Yf0 = np.array([t0 ** (a + 1) for a in range(F)])[:, None] * f[0]
        L0, d0 = factor_pinned(TL, pin[0])
        z = np.zeros((F, D))
        for d in range(D):
            rhs = hn * (P[1, d] - P[0, d])
            rhs += TL[:, [k for k in range(F) if pin[0][k]]] @ Yf0[[k for k in range(F) if pin[0][k]], d]
            nxt = np.array([t0 ** (b + 1) * f[1, b, d] if pin[1][b] else 0.0 for b in range(F)])
            rhs += BL.T @ nxt
            zz = solve(L0, d0, -rhs)
            for k in range(F):
                if pin[0][k]:
                    zz[k] = Yf0[k, d]
            z[:, d] = zz
        Ls.append(L0), Ds.append(d0), Zs.append(z)
        for J in range(1, KC + 1):
            Lp, Dp, zp = Ls[-1], Ds[-1], Zs[-1]
            W = np.linalg.solve(Lp, BL.T)      # L^-1 BL~^T, [k][a]
            Pm = BR - W.T @ np.diag(Dp) @ W
            if J < KC:
                rho = T[J - 1] / T[J]
                e = np.array([[rho ** (a + b + 3 - 2 * R) for b in range(F)] for a in range(F)])
                S = TL + e * Pm
                Lc, dc = factor_pinned(S, pin[J])
                z = np.zeros((F, D))
                YfJ = np.array([T[J] ** (a + 1) for a in range(F)])[:, None] * f[J]
                for d in range(D):
                    qv = hp * (P[J, d] - P[J - 1, d]) + BL @ zp[:, d]
                    rhs = np.array([rho ** (a + 2 - 2 * R) for a in range(F)]) * qv + hn * (P[J + 1, d] - P[J, d])
                    own = (TL + e * BR) @ np.array([YfJ[k, d] if pin[J][k] else 0.0 for k in range(F)])
                    nxt = BL.T @ np.array([T[J] ** (b + 1) * f[J + 1, b, d] if pin[J + 1][b] else 0.0
                                           for b in range(F)])
                    zz = solve(Lc, dc, -(rhs + own + nxt))
                    for k in range(F):
                        if pin[J][k]:
                            zz[k] = YfJ[k, d]
                    z[:, d] = zz
                Ls.append(Lc), Ds.append(dc), Zs.append(z)
            else:  # the meeting vertex: this chain's half in the unscaled basis
                Tm = T[KC - 1]
                Sh = np.array([[Tm ** (a + b + 3 - 2 * R) * Pm[a, b] for b in range(F)] for a in range(F)])
                rh = np.zeros((F, D))
                for d in range(D):
                    qv = hp * (P[J, d] - P[J - 1, d]) + BL @ zp[:, d]
                    own = np.array([sum(Tm ** (a + k + 3 - 2 * R) * BR[a, k] * f[J, k, d]
                                        for k in range(F) if pin[J][k]) for a in range(F)])
                    rh[:, d] = -(np.array([Tm ** (a + 2 - 2 * R) for a in range(F)]) * qv + own)
                halves[ch] = (Sh, rh)
        st[ch] = (Ls, Ds, Zs, v, m, T, pin, f, P)
    # merge: partner half in this chain's coordinates, (-1)^(a+b) / (-1)^(a+1)
    sg = np.array([[(-1.0) ** (a + b) for b in range(F)] for a in range(F)])
    sr = np.array([(-1.0) ** (a + 1) for a in range(F)])
    xm = {}
    for ch in (0, 1):
        S = halves[ch][0] + sg * halves[1 - ch][0]
        rhs = halves[ch][1] + sr[:, None] * halves[1 - ch][1]
        pin = st[ch][6]
        Lm, dm = factor_pinned(S, pin[KC])
        x = np.stack([solve(Lm, dm, rhs[:, d]) for d in range(D)], axis=1)
        for k in range(F):
            if pin[KC][k]:
                x[k] = st[ch][7][KC, k]
        xm[ch] = x
    # backward, coefficients per chain segment
    A1 = a1inv(N)
    coeffs = np.zeros((K, D, N))
    for ch in (0, 1):
        Ls, Ds, Zs, v, m, T, pin, f, P = st[ch]
        Tm = T[KC - 1]
        Y = xm[ch] * np.array([Tm ** (a + 1) for a in range(F)])[:, None]  # scaled with T_{KC-1}
        Tn = Tm
        for J in range(KC - 1, -1, -1):
            rho = T[J] / Tn
            vfull = Y * np.array([rho ** (b + 1) for b in range(F)])[:, None]
            vm = vfull * np.array([0.0 if pin[J + 1][b] else 1.0 for b in range(F)])[:, None]
            y = np.zeros((F, D))
            for d in range(D):
                tt = solve(Ls[J], Ds[J], BL.T @ vm[:, d])
                y[:, d] = Zs[J][:, d] - tt
            # segment J (chain), scaled end values y (start) / vfull (end)
            seg = J if ch == 0 else K - 1 - J
            for d in range(D):
                sh = np.zeros(N)
                if ch == 0:
                    sh[1:H] = y[:, d]
                    sh[H + 1:] = vfull[:, d]
                    sh[H] = P[J + 1, d] - P[J, d]
                    p0 = P[J, d]
                else:  # back to the original direction: odd derivatives negated
                    sgn = np.array([(-1.0) ** (a + 1) for a in range(F)])
                    sh[1:H] = sgn * vfull[:, d]
                    sh[H + 1:] = sgn * y[:, d]
                    sh[H] = P[J, d] - P[J + 1, d]
                    p0 = P[J + 1, d]
                c = (A1 @ sh) * np.array([T[J] ** (-j) for j in range(N)])
                c[0] = p0
                coeffs[seg, d] = c
            Y, Tn = y, T[J]
    return coeffs


def main():
    from oracle import pyoracle
    import mav_trajectory_generation_cmake_amd as mtg
    N, K, R, trials = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (10, 10, 4, 40)))
    H = N // 2
    vals, mask, times = mtg.random_vertices_path_batch(N, 3, K, trials, seed0=11, max_derivative=min(4, H - 1))
    rng = np.random.default_rng(3)
    mask = mask.copy()
    vals = vals.copy()
    for b in range(trials):  # random extra pins / unpins, positions always fixed
        mask[b] = (rng.integers(0, 1 << H, size=K + 1) | 1).astype(np.uint8)
        vals[b, :, 1:, :] = rng.normal(size=vals[b, :, 1:, :].shape)
    ref = pyoracle.solve_linear_batch(N, R, vals, mask.astype(np.uint32), times)
    worst = 0.0
    for b in range(trials):
        c = emulate(N, R, vals[b], mask[b], times[b])
        tp = np.power(times[b][:, None, None], np.arange(N))
        err = np.max(np.abs(c - ref[b]) * tp) / np.max(np.abs(ref[b]) * tp)
        worst = max(worst, err)
    print("N=%d K=%d R=%d: %d trajectories with random masks, worst scale-normalised error vs oracle %.2e"
          % (N, K, R, trials, worst))
    assert worst < 1e-6


if __name__ == "__main__":
    main()
