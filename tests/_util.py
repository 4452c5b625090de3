"""Shared helpers for the parity tests (fixtures, layouts, error metrics)."""
import glob
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_cases():
    """The truth fixtures (tests/golden/make_golden.py); host_solve_bitwise.npz and
    config4_truth_sample.npz are fixtures of their own (tests/golden/make_host_fixture.py,
    tests/golden/make_config4_truth.py)."""
    own = ("host_solve_bitwise.npz", "config4_truth_sample.npz")
    return sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                  if os.path.basename(p) not in own)


def load_golden(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def to_abi(values_nd, mask32, N):
    """[B][V][nd][D] generator layout -> ABI values [B][V][N/2][D], uint8 mask (bits >= 7 folded into bit 7)."""
    h = N // 2
    B, V, nd, D = values_nd.shape
    vals = np.zeros((B, V, h, D))
    k = min(h, nd)
    vals[:, :, :k, :] = values_nd[:, :, :k, :]
    m = mask32.astype(np.uint32)
    m8 = (m & 0x7F) | np.where(m >> 7, 0x80, 0)
    return vals, m8.astype(np.uint8)


def scale_normalised_error(c, ref, times):
    """max over (traj, segment, dim) of max_k |c_k - ref_k| T^k / max_k |ref_k| T^k.

    The recommended tolerance metric of SURVEY.md 8(c): coefficient k of a
    segment of duration T contributes c_k T^k to the position at the segment
    end, so this is the relative error of the polynomial over its own domain."""
    c = np.asarray(c)
    ref = np.asarray(ref)
    N = c.shape[-1]
    tp = np.power(np.asarray(times)[..., None], np.arange(N))  # [B][K][N]
    tp = tp[..., None, :]  # [B][K][1][N]
    err = np.abs(c - ref) * tp
    scale = np.max(np.abs(ref) * tp, axis=-1)
    scale = np.where(scale == 0, 1.0, scale)
    return float(np.max(np.max(err, axis=-1) / scale))


def masked_elementwise_rel(c, ref, times, floor=1e-12):
    """Element-wise relative error on coefficients with |ref_k| T^k >= floor * scale."""
    N = c.shape[-1]
    tp = np.power(np.asarray(times)[..., None], np.arange(N))[..., None, :]
    mag = np.abs(ref) * tp
    scale = np.max(mag, axis=-1, keepdims=True)
    sel = mag >= floor * scale
    rel = np.abs(c - ref) / np.where(np.abs(ref) > 0, np.abs(ref), 1.0)
    return float(np.max(np.where(sel, rel, 0.0)))


def base_coefficient(n, i):
    if i < n:
        return 0.0
    out = 1.0
    for k in range(i - n + 1, i + 1):
        out *= k
    return out


def poly_eval(c, t, derivative=0):
    """Vectorised Polynomial::evaluate (polynomial.h:138-151) over trailing coefficient axis."""
    c = np.asarray(c)
    N = c.shape[-1]
    if derivative >= N:
        return np.zeros(c.shape[:-1])
    row = np.array([base_coefficient(derivative, j) for j in range(N)])
    res = row[N - 1] * c[..., N - 1]
    for j in range(N - 2, derivative - 1, -1):
        res = res * t + row[j] * c[..., j]
    return res


def check_path(values, mask, times, coeffs, N, relative=False):
    """Vectorised checkPath (test/test_polynomial_optimization.cpp:73-131) over a batch.

    Fixed constraints met at segment ends, derivatives 0..N/2-1 continuous at
    interior vertices.  Returns the worst absolute violation (the reference
    asserts < 1e-6, :75), or with relative=True the violation divided by
    max(1, largest |derivative k| at the trajectory's vertices) -- needed for the
    bench generator, whose U(0, 10) segment lengths produce millisecond segments
    with derivatives of 1e8 and more (the reference path itself misses 1e-6
    absolute there)."""
    h = N // 2
    B, V, _, D = values.shape
    K = V - 1
    T = times[:, :, None]  # [B][K][1]
    worst = 0.0
    for k in range(h):
        start = poly_eval(coeffs, np.zeros_like(T), k)  # [B][K][D]
        end = poly_eval(coeffs, T, k)  # [B][K][D]
        fixed = ((mask[:, :, None] >> k) & 1).astype(bool)  # [B][V][1]
        want = values[:, :, k, :]  # [B][V][D]
        # at t=0 of segment i: vertex i; at t=T of segment i: vertex i+1
        if relative:
            scale = np.maximum(1.0, np.maximum(np.abs(start).max(axis=(1, 2)), np.abs(end).max(axis=(1, 2))))
            scale = scale[:, None, None]
        else:
            scale = 1.0
        e0 = np.abs(start - want[:, :K]) / scale
        e1 = np.abs(end - want[:, 1:]) / scale
        worst = max(worst, float(np.max(np.where(fixed[:, :K], e0, 0.0))),
                    float(np.max(np.where(fixed[:, 1:], e1, 0.0))))
        if K > 1:
            cont = np.abs(end[:, :-1] - start[:, 1:]) / (scale if relative else 1.0)
            worst = max(worst, float(np.max(cont)))
    return worst
