"""Shared helpers for the parity tests (fixtures, layouts, error metrics)."""
import glob
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_cases():
    """The truth fixtures (tests/golden/make_golden.py); host_solve_bitwise.npz, the truth samples
    config4_truth_sample.npz / accel12_truth_sample.npz and offpattern_truth_n12.npz are fixtures of
    their own (tests/golden/make_host_fixture.py, make_config4_truth.py, make_offpattern_truth.py)."""
    own = ("host_solve_bitwise.npz", "config4_truth_sample.npz", "accel12_truth_sample.npz", "offpattern_truth_n12.npz")
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


def off_pattern_batch(N, D, K, B, seed0, kind):
    """Batches whose masks are not the reference generators' pattern (the DL kernel's other passes):
    "accel" / "jerk" are createRandomVertices with the ends fixed only to ACCELERATION / JERK (the
    reference's 2_vertices_rand and ConstraintPacking masks, test/test_polynomial_optimization.cpp:747-774,
    :777-836: the ends pass); "ends" pins random subsets of derivatives 1..N/2-1 at the two end
    vertices only (ends pass); "random" pins derivatives 1..N/2-1 at random per vertex (values random)
    and "vel" adds a fixed velocity at every interior vertex (the general-mask pass); "mixed" mixes the
    pattern, "random", "ends" and a free interior position (the fallback)."""
    from mav_trajectory_generation_cmake_amd import random_vertices_batch, random_vertices_path_batch
    h = N // 2
    rng = np.random.default_rng(seed0)
    if kind in ("accel", "jerk"):
        md = min(2 if kind == "accel" else 3, h - 1)
        return random_vertices_batch(N, D, K, B, [-50.0] * D, [50.0] * D, seed0=seed0, max_derivative=md)
    vals, mask, times = random_vertices_path_batch(N, D, K, B, seed0=seed0, max_derivative=min(4, h - 1))
    vals, mask = vals.copy(), mask.copy()
    if kind == "vel":
        mask[:, 1:-1] |= 2
        vals[:, 1:-1, 1, :] = rng.normal(size=vals[:, 1:-1, 1, :].shape)
    elif kind in ("random", "mixed", "ends"):
        sel = rng.random(B) < (1.0 if kind == "random" else (0.5 if kind == "mixed" else 0.0))
        pins = (rng.integers(0, 1 << h, size=(B, K + 1)) | 1).astype(np.uint8)
        mask[sel] = pins[sel]
        vals[sel, :, 1:, :] = rng.normal(size=vals[sel, :, 1:, :].shape)
        ends = ~sel & (rng.random(B) < (1.0 if kind == "ends" else 0.5))
        for v in (0, K):
            mask[ends, v] = pins[ends, v]
            vals[ends, v, 1:, :] = rng.normal(size=vals[ends, v, 1:, :].shape)
        if kind == "mixed":
            free_pos = rng.random(B) < 0.05
            mask[free_pos, K // 2] &= np.uint8(0xFE)  # a free interior position: the fallback
    return vals, mask, times
