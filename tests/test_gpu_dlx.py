"""The long-chain dimension-lane kernel (round 6, mtg_solve_dlx.inc): N = 6..12
trajectories whose K has no fixed-length DL kernel and no column kernel -- the reference benchmark's
K = 50 and 100 (src/polynomial_timing_evaluation.cpp:117) among them.

The kernel serves the trajectories whose interior vertices fix exactly their position (any pins at the
two end vertices); the others run the general kernel's block function (solve_dlx_rest_kernel) and
must come out bit for bit as the general kernel's.  Parity: against the general kernel (two FP64
orderings of the same block-tridiagonal solve) and the oracle (the reference algorithm restated,
1e-6 scale-normalised, north_star's tolerance), with 60-digit truth arbitrating where the orderings
differ, plus checkPath's invariants (test/test_polynomial_optimization.cpp:73-131).
"""
import os
import sys

import numpy as np
import pytest

from _util import check_path, off_pattern_batch, scale_normalised_error

pytestmark = pytest.mark.gpu

ORACLE_TOL = 1e-6
# DLX against the general kernel: two FP64 orderings; the scaled basis keeps the recurrence's numbers
# O(1), the general kernel's unscaled pivots span T^(3-2r) .. T^(N-1-2r).  Where they differ by more
# than PAIR_TOL the shorter shapes are arbitrated by 60-digit truth.
PAIR_TOL = 1e-8


def _oracle():
    from oracle import pyoracle
    return pyoracle


def _kernel(N, D, K, r, B):
    from mav_trajectory_generation_cmake_amd import _native as nat
    return nat.solve_kernel(N, D, K, r, B=B)


def nat_traj_bad_time():
    from mav_trajectory_generation_cmake_amd import _native as nat
    return nat.MTG_TRAJ_BAD_TIME


def _served(mask, K):
    """Trajectories the DLX kernel itself solves: interior masks exactly 1 (the position), end masks with bit 0."""
    ends = (mask[:, 0] & 1).astype(bool) & (mask[:, K] & 1).astype(bool)
    interior = np.all(mask[:, 1:K] == 1, axis=1) if K > 1 else np.ones(len(mask), bool)
    return ends & interior


def _batch(N, D, K, B, seed0, kind):
    if kind == "pattern" and N == 12 and D == 1:
        # config 4's generator (createRandomVertices(SNAP, ...) + estimateSegmentTimes(3, 5)): the path
        # generator's millisecond segments next to 18-s ones leave some N = 12 problems beyond FP64
        # (both kernels 1e-2 .. 1 from truth)
        from mav_trajectory_generation_cmake_amd import random_vertices_batch
        return random_vertices_batch(N, D, K, B, [-10.0] * D, [10.0] * D, seed0=seed0, max_derivative=4,
                                     v_max=3.0, a_max=5.0)
    if kind == "pattern":
        from mav_trajectory_generation_cmake_amd import random_vertices_path_batch
        return random_vertices_path_batch(N, D, K, B, seed0=seed0, max_derivative=min(4, N // 2 - 1))
    return off_pattern_batch(N, D, K, B, seed0, kind)


def _compare_general(N, r, vals, mask, times, x, g, far_limit=8):
    """x (default path: DLX) against g (the general kernel): status, n_free equal; the trajectories DLX
    does not serve bit for bit; the others within PAIR_TOL, or -- for at most far_limit of them --
    arbitrated by 60-digit truth (make_golden.truth_solve_banded): DLX within 1e-9 of truth, at least
    as close to it as the general kernel, or (ill-conditioned problems) closer to it than the reference
    algorithm and within 4x of the best FP64 solve; free values and cost within 1e-8 (relative to the general
    kernel's, except on the arbitrated trajectories)."""
    K = times.shape[1]
    B = len(times)
    np.testing.assert_array_equal(x["status"], g["status"])
    np.testing.assert_array_equal(x["n_free"], g["n_free"])
    rest = ~_served(mask, K)
    for k in ("coeffs", "free", "cost"):
        np.testing.assert_array_equal(x[k][rest], g[k][rest], err_msg="rest kernel " + k)
    # (a NOT_SPD trajectory -- both kernels flag the same ones -- has no meaningful solution to compare)
    ok = x["status"] & 0xFF == 0
    dg = np.array([scale_normalised_error(x["coeffs"][b:b + 1], g["coeffs"][b:b + 1], times[b:b + 1]) if ok[b]
                   else 0.0 for b in range(B)])
    far = np.nonzero(dg > PAIR_TOL)[0]
    assert len(far) <= far_limit, (len(far), np.sort(dg)[-10:])
    if len(far):
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
        from make_golden import fp64_best_solve, truth_solve_banded
        for b in far:
            sl = slice(b, b + 1)
            tr = truth_solve_banded(N, r, vals[b], mask[b], times[b])[None]
            e_x = scale_normalised_error(x["coeffs"][sl], tr, times[sl])
            e_g = scale_normalised_error(g["coeffs"][sl], tr, times[sl])
            if e_x <= max(1e-9, e_g):
                continue
            # an ill-conditioned problem (segment times spanning two decades): closer to truth than the
            # reference algorithm (the oracle) and within 4x of the best FP64 solve (make_golden)
            ref = _oracle().solve_linear_batch(N, r, vals[sl], mask[sl].astype(np.uint32), times[sl])
            e_ref = scale_normalised_error(ref, tr, times[sl])
            e_best = scale_normalised_error(fp64_best_solve(N, r, vals[b], mask[b], times[b])[None], tr, times[sl])
            assert e_x <= e_ref and e_x <= 4.0 * e_best, (int(b), e_x, e_g, e_ref, e_best, dg[b])
    near = ok.copy()
    near[far] = False
    nf = int(np.max(x["n_free"]))
    fscale = np.max(np.abs(g["free"][near, :, :nf]), axis=-1, keepdims=True) + 1.0
    assert np.max(np.abs(x["free"][near, :, :nf] - g["free"][near, :, :nf]) / fscale) <= 1e-8
    assert np.max(np.abs(x["cost"][near] - g["cost"][near]) / (np.abs(g["cost"][near]) + 1.0)) <= 1e-8
    return dg


def _check_path_vs_general(N, vals, mask, times, x, g):
    """checkPath's invariants (fixed values reproduced, continuity across vertices, relative to the
    segment's scale) within 1e-6 or, where the problem's own conditioning puts the general kernel's
    solve above that (r = 2 over 50 segments: ~5e-6), within 2x of the general kernel's."""
    ok = x["status"] & 0xFF == 0
    cx = check_path(vals[ok], mask[ok], times[ok], x["coeffs"][ok], N, relative=True)
    cg = check_path(vals[ok], mask[ok], times[ok], g["coeffs"][ok], N, relative=True)
    assert cx <= max(1e-6, 2.0 * cg), (cx, cg)


def _vs_oracle_and_truth(N, r, vals, mask, times, coeffs, S, T=3):
    """The first S trajectories against the oracle at north_star's 1e-6 (N = 10 with SNAP, r = 4: the
    configs' objective), and the first T against 60-digit truth: within 1e-9, or closer to it than the
    reference algorithm (which is ~1e-5 off at r = 1 or N = 12)."""
    O = _oracle()
    if N == 10 and r == 4:
        ref = O.solve_linear_batch(N, r, vals[:S], mask[:S].astype(np.uint32), times[:S], threads=8)
        assert scale_normalised_error(coeffs[:S], ref, times[:S]) <= ORACLE_TOL
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_golden import truth_solve_banded
    for b in range(T):
        sl = slice(b, b + 1)
        tr = truth_solve_banded(N, r, vals[b], mask[b], times[b])[None]
        e_x = scale_normalised_error(coeffs[sl], tr, times[sl])
        if e_x <= 1e-9:
            continue
        ref = O.solve_linear_batch(N, r, vals[sl], mask[sl].astype(np.uint32), times[sl])
        e_ref = scale_normalised_error(ref, tr, times[sl])
        assert e_x <= e_ref, (b, e_x, e_ref)


SHAPES = [(10, 3, 50, 4), (10, 3, 100, 4), (10, 3, 11, 4), (10, 3, 13, 4), (10, 1, 50, 2), (10, 4, 37, 3),
          (10, 2, 64, 4), (10, 3, 12, 1), (12, 3, 21, 3), (12, 3, 40, 3), (12, 4, 33, 2), (12, 1, 25, 4),
          (8, 3, 30, 3), (8, 2, 13, 2), (8, 4, 51, 1), (6, 3, 40, 2), (6, 1, 17, 1)]


@pytest.mark.parametrize("N,D,K,r", SHAPES)
def test_dlx_pattern_vs_general_and_oracle(gpu_ctx, N, D, K, r):
    """The reference generators' pattern (createRandomVerticesPath, ends to SNAP -- N = 12: derivatives
    0..4 at the ends, the fifth free): DLX against the general kernel and, for the first trajectories,
    the oracle (N = 10; N = 12's FP64 reference algorithm is itself ~1e-5 from truth at these K)."""
    B = 437 if K <= 64 else 131  # ragged: not a multiple of the trajectories per wave
    vals, mask, times = _batch(N, D, K, B, 3100 + K + D, "pattern")
    assert _kernel(N, D, K, r, B) == "solve_dlx_kernel"
    kw = dict(free=True, n_free=True, cost=True, status=True)
    x = gpu_ctx.solve_linear_batch(N, r, vals, mask, times, **kw)
    g = gpu_ctx.solve_linear_batch(N, r, vals, mask, times, general=True, **kw)
    # (N = 12 with r = 5 over a 7-ms segment: NOT_SPD in both kernels, lin_impl's Q of T^(1-2r) overflows
    # the pivots' range -- one trajectory of this batch)
    assert np.mean(x["status"] == 0) >= 0.99 and np.all(x["status"] & 0xFF != nat_traj_bad_time())
    _compare_general(N, r, vals, mask, times, x, g)
    _check_path_vs_general(N, vals, mask, times, x, g)
    ok = np.nonzero(x["status"] == 0)[0]
    _vs_oracle_and_truth(N, r, vals[ok], mask[ok], times[ok], x["coeffs"][ok], 24 if K <= 64 else 6)


@pytest.mark.parametrize("N,D,K,r,kind", [(10, 3, 50, 4, "accel"), (10, 3, 50, 4, "jerk"), (10, 3, 50, 4, "ends"),
                                          (10, 3, 50, 4, "mixed"), (10, 3, 50, 4, "vel"), (10, 3, 50, 4, "random"),
                                          (10, 3, 17, 4, "mixed"), (10, 1, 23, 2, "ends"), (12, 3, 30, 3, "accel"),
                                          (12, 4, 30, 3, "mixed"), (12, 3, 21, 3, "ends"), (8, 3, 30, 3, "accel"),
                                          (8, 3, 25, 3, "mixed"), (6, 2, 20, 2, "ends")])
def test_dlx_other_masks(gpu_ctx, N, D, K, r, kind):
    """Masks other than the generators' pattern: ends fixed only to ACCELERATION / JERK (2_vertices_rand,
    ConstraintPacking, test/test_polynomial_optimization.cpp:747-836) and random end pins -- DLX's
    run-time end pins --, and interior pins / free positions ("vel", "random", "mixed") -- the rest
    kernel, bit for bit the general kernel's."""
    B = 437
    vals, mask, times = _batch(N, D, K, B, 5200 + K + D, kind)
    assert _kernel(N, D, K, r, B) == "solve_dlx_kernel"
    kw = dict(free=True, n_free=True, cost=True, status=True)
    x = gpu_ctx.solve_linear_batch(N, r, vals, mask, times, **kw)
    g = gpu_ctx.solve_linear_batch(N, r, vals, mask, times, general=True, **kw)
    assert np.all(x["status"] == 0)
    served = _served(mask, K)
    if kind in ("vel", "random"):
        assert not served.any()
    elif kind in ("accel", "jerk", "ends"):
        assert served.all()
    _compare_general(N, r, vals, mask, times, x, g)
    _check_path_vs_general(N, vals, mask, times, x, g)
    _vs_oracle_and_truth(N, r, vals, mask, times, x["coeffs"], 24)


@pytest.mark.parametrize("K", [50, 100])
def test_dlx_full_size(gpu_ctx, K):
    """1e4 trajectories of the reference benchmark's shape (createRandomVerticesPath, N = 10, D = 3,
    SNAP; K = 50 / 100): every trajectory against the general kernel, checkPath on all, and a sample
    against the oracle."""
    N, D, r, B = 10, 3, 4, 10000
    from mav_trajectory_generation_cmake_amd import random_vertices_path_batch
    vals, mask, times = random_vertices_path_batch(N, D, K, B, seed0=K * 1000)
    assert _kernel(N, D, K, r, B) == "solve_dlx_kernel"
    kw = dict(free=True, n_free=True, cost=True, status=True)
    x = gpu_ctx.solve_linear_batch(N, r, vals, mask, times, **kw)
    g = gpu_ctx.solve_linear_batch(N, r, vals, mask, times, general=True, **kw)
    assert np.all(x["status"] == 0)
    _compare_general(N, r, vals, mask, times, x, g, far_limit=30)
    _check_path_vs_general(N, vals, mask, times, x, g)
    idx = np.random.default_rng(K).choice(B, 8, replace=False)
    _vs_oracle_and_truth(N, r, vals[idx], mask[idx], times[idx], x["coeffs"][idx], 8)


@pytest.mark.parametrize("N,D,K,r", [(10, 3, 50, 4), (12, 3, 21, 3)])
def test_dlx_result_independent_of_batch_composition(gpu_ctx, N, D, K, r):
    """A trajectory's bits do not depend on the call it is in: the whole batch (8% of trajectories with
    a fixed interior velocity -- the rest kernel's), reversed, in chunks of 37 and 300, and single
    trajectories give the same coefficients, free values, cost and status."""
    from mav_trajectory_generation_cmake_amd import random_vertices_path_batch
    B = 700
    vals, mask, times = random_vertices_path_batch(N, D, K, B, seed0=8800, max_derivative=min(4, N // 2 - 1))
    rng = np.random.default_rng(6)
    odd = rng.random(B) < 0.08
    for b in np.nonzero(odd)[0]:
        mask[b, 1 + int(rng.integers(0, K - 1))] |= np.uint8(2)
    kw = dict(free=True, cost=True, status=True)
    whole = gpu_ctx.solve_linear_batch(N, r, vals, mask, times, **kw)
    assert np.all(whole["status"] == 0)
    keys = ("coeffs", "free", "cost", "status")
    rev = gpu_ctx.solve_linear_batch(N, r, vals[::-1].copy(), mask[::-1].copy(), times[::-1].copy(), **kw)
    for k in keys:
        np.testing.assert_array_equal(rev[k][::-1], whole[k], err_msg="reversed " + k)
    for chunk in (37, 300):
        for s0 in range(0, B, chunk):
            part = gpu_ctx.solve_linear_batch(N, r, vals[s0:s0 + chunk], mask[s0:s0 + chunk], times[s0:s0 + chunk], **kw)
            for k in keys:
                np.testing.assert_array_equal(part[k], whole[k][s0:s0 + chunk], err_msg="chunk %d %s" % (chunk, k))
    for b in list(np.nonzero(odd)[0][:2]) + [0, B - 1]:
        one = gpu_ctx.solve_linear_batch(N, r, vals[b:b + 1], mask[b:b + 1], times[b:b + 1], **kw)
        for k in keys:
            np.testing.assert_array_equal(one[k], whole[k][b:b + 1], err_msg="single %d %s" % (b, k))


def test_dlx_status_codes(gpu_ctx):
    """Bad, tiny and huge segment times and dropped orders at the end vertices set the general kernel's
    status bits (lin_impl:287 CHECK_GT, polynomial.h:225, lin_impl:84-87)."""
    from mav_trajectory_generation_cmake_amd import _native as nat
    N, D, K, r, B = 10, 3, 50, 4, 40
    vals, mask, times = _batch(N, D, K, B, 77, "pattern")
    t = times.copy()
    t[3, 2] = 0.0
    t[4, 40] = 1e-17
    t[5, :] = 1e200
    t[6, 30] = -1.0
    t[7, 49] = np.nan
    m = mask.copy()
    m[8, 0] |= np.uint8(0x40)  # an order above N/2 - 1 at an end vertex: dropped, WARN_DROPPED
    m[9, K] |= np.uint8(0x20)
    kw = dict(status=True)
    x = gpu_ctx.solve_linear_batch(N, r, vals, m, t, **kw)
    g = gpu_ctx.solve_linear_batch(N, r, vals, m, t, general=True, **kw)
    np.testing.assert_array_equal(x["status"], g["status"])
    assert x["status"][3] & nat.MTG_TRAJ_BAD_TIME and x["status"][6] & nat.MTG_TRAJ_BAD_TIME
    assert x["status"][7] & nat.MTG_TRAJ_BAD_TIME
    assert x["status"][4] & nat.MTG_TRAJ_NOT_SPD and not x["status"][4] & nat.MTG_TRAJ_BAD_TIME
    assert x["status"][5] & nat.MTG_TRAJ_NOT_SPD
    assert x["status"][8] == nat.MTG_TRAJ_WARN_DROPPED and x["status"][9] == nat.MTG_TRAJ_WARN_DROPPED
    ok = np.ones(B, bool)
    ok[3:10] = False
    assert np.all(x["status"][ok] == 0)
    # the dropped orders change nothing else
    clean = gpu_ctx.solve_linear_batch(N, r, vals, mask, times)
    y = gpu_ctx.solve_linear_batch(N, r, vals, m, times)
    np.testing.assert_array_equal(y["coeffs"][8:10], clean["coeffs"][8:10])


def test_dlx_time_sweep(gpu_ctx):
    """The sweep (trajectory x candidate pairs, scaled times, mtg_time_sweep_batch) on DLX: each
    candidate's cost equals a solve at the scaled times on the same kernel, and the general kernel's
    sweep within 1e-8."""
    N, D, K, r, B = 10, 3, 50, 4, 60
    vals, mask, times = _batch(N, D, K, B, 901, "pattern")
    scales = 0.5 + np.arange(16) / 15.0
    assert _kernel(N, D, K, r, B * len(scales)) == "solve_dlx_kernel"
    J = gpu_ctx.time_sweep_batch(N, r, vals, mask, times, scales)
    Jg = gpu_ctx.time_sweep_batch(N, r, vals, mask, times, scales, general=True)
    np.testing.assert_allclose(J, Jg, rtol=1e-8)
    for ci in (0, 7, 15):
        ref = gpu_ctx.solve_linear_batch(N, r, vals, mask, times * scales[ci], cost=True)["cost"]
        np.testing.assert_allclose(J[:, ci], ref, rtol=1e-12, atol=0)


def test_dlx_output_alignment_and_device_pointers(gpu_ctx):
    """An output array only 8-B aligned (the AL16 = 0 instantiation) and device-pointer calls give the
    host-array call's coefficients bit for bit (a "mixed" batch: DLX and rest kernel)."""
    import torch
    N, D, K, r, B = 10, 3, 50, 4, 123
    vals, mask, times = _batch(N, D, K, B, 4242, "mixed")
    dev = torch.device("cuda:0")
    dv, dm, dt = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (vals, mask, times))
    shape = (B, K, D, N)
    c16 = torch.zeros(shape, dtype=torch.float64, device=dev)
    buf = torch.full((B * K * D * N + 1,), np.nan, dtype=torch.float64, device=dev)
    c8 = buf[1:].view(shape)
    assert c8.data_ptr() % 16 == 8
    gpu_ctx.solve_linear_batch(N, r, dv, dm, dt, coeffs=c16)
    gpu_ctx.solve_linear_batch(N, r, dv, dm, dt, coeffs=c8)
    torch.cuda.synchronize()
    host = gpu_ctx.solve_linear_batch(N, r, vals, mask, times)["coeffs"]
    np.testing.assert_array_equal(c16.cpu().numpy(), host)
    np.testing.assert_array_equal(c8.cpu().numpy(), host)
    assert np.isnan(buf[0].item())


def test_dlx_pipelined_host_arrays(gpu_ctx):
    """A host-array batch above the pipeline threshold (chunks on several streams, a workspace per
    slot) equals the device-resident solve bit for bit."""
    import torch
    N, D, K, r, B = 10, 3, 100, 4, 3000
    from mav_trajectory_generation_cmake_amd import random_vertices_path_batch
    vals, mask, times = random_vertices_path_batch(N, D, K, B, seed0=31)
    host = gpu_ctx.solve_linear_batch(N, r, vals, mask, times, status=True)
    assert np.all(host["status"] == 0)
    dev = torch.device("cuda:0")
    dv, dm, dt = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (vals, mask, times))
    c = torch.zeros((B, K, D, N), dtype=torch.float64, device=dev)
    gpu_ctx.solve_linear_batch(N, r, dv, dm, dt, coeffs=c)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(c.cpu().numpy(), host["coeffs"])
