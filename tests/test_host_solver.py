"""The library's host solve path (mtg_host_solve_linear_batch, csrc/mtg_host_solve.cpp): the same
algorithm as the HIP kernels in scalar C++, used by the drop-in PolynomialOptimization<N> for
single problems (BASELINE config 1, "on CPU").  CPU tests: against the 60-digit truth fixtures and
the oracle (the restated reference algorithm), with the GPU parity tests' tolerances."""
import numpy as np
import pytest

from _util import (check_path, golden_cases, load_golden, masked_elementwise_rel, scale_normalised_error,
                   to_abi)

import mav_trajectory_generation_cmake_amd as mtg
from mav_trajectory_generation_cmake_amd import _native as nat

TRUTH_TOL = 1e-9
ORACLE_TOL_N10 = 1e-6


def _oracle():
    from oracle import pyoracle
    return pyoracle


@pytest.mark.parametrize("case", golden_cases())
def test_golden_truth(case):
    g = load_golden(case)
    N, r = int(g["N"]), int(g["r"])
    vals, mask = to_abi(g["values"], g["mask"], N)
    out = mtg.host_solve_linear_batch(N, r, vals, mask, g["times"], free=True, n_free=True, cost=True, status=True)
    assert np.all(out["status"] & 0xFF == 0), out["status"]
    assert scale_normalised_error(out["coeffs"], g["coeffs"], g["times"]) <= TRUTH_TOL, case
    assert masked_elementwise_rel(out["coeffs"], g["coeffs"], g["times"], floor=1e-4) <= 1e-6, case
    np.testing.assert_array_equal(out["n_free"], g["n_free"])
    assert np.max(np.abs(out["cost"] - g["cost"]) / np.maximum(np.abs(g["cost"]), 1e-300)) <= 1e-9
    for b in range(len(out["n_free"])):
        nf = int(g["n_free"][b])
        if nf:
            ref = g["free"][b][:, :nf]
            scale = np.maximum(np.max(np.abs(ref), axis=1, keepdims=True), 1e-300)
            assert np.max(np.abs(out["free"][b][:, :nf] - ref) / scale) <= 1e-7, case
            assert np.all(out["free"][b][:, nf:] == 0.0)


@pytest.mark.parametrize("K", [1, 2, 3, 5, 9, 10, 12, 13, 20, 50, 100])
def test_segment_counts_vs_oracle(K):
    """The reference bench's K in {2, 10, 50, 100} (src/polynomial_timing_evaluation.cpp:117) and the
    GPU kernels' bucket edges."""
    O = _oracle()
    vals, mask, times = mtg.random_vertices_path_batch(10, 3, K, 16, seed0=77)
    out = mtg.host_solve_linear_batch(10, 4, vals, mask, times, status=True, cost=True)
    assert np.all(out["status"] == 0)
    ref = O.solve_linear_batch(10, 4, vals, mask.astype(np.uint32), times)
    assert scale_normalised_error(out["coeffs"], ref, times) <= ORACLE_TOL_N10
    assert check_path(vals, mask, times, out["coeffs"], 10, relative=True) < 1e-8


def test_mixed_masks_vs_oracle():
    """Per-problem masks with extra fixed derivatives at interior vertices (any pattern)."""
    O = _oracle()
    B = 64
    vals, mask, times = mtg.random_vertices_batch(10, 3, 7, B, [-10, -20, -10], [10, 20, 10], seed0=9)
    rng = np.random.default_rng(5)
    mask = mask.copy()
    mask[:, 1:-1] |= (rng.integers(0, 32, size=mask[:, 1:-1].shape) & 0x1E).astype(np.uint8)
    vals = vals + rng.normal(size=vals.shape) * (mask[:, :, None, None] > 0)
    out = mtg.host_solve_linear_batch(10, 4, vals, mask, times, status=True)
    assert np.all(out["status"] == 0)
    ref = O.solve_linear_batch(10, 4, vals, mask.astype(np.uint32), times)
    assert scale_normalised_error(out["coeffs"], ref, times) <= ORACLE_TOL_N10
    assert check_path(vals, mask, times, out["coeffs"], 10, relative=True) < 1e-8


@pytest.mark.parametrize("N,D,r", [(4, 1, 1), (6, 2, 2), (8, 3, 3), (12, 4, 5), (12, 3, 0)])
def test_other_shapes_vs_oracle(N, D, r):
    O = _oracle()
    vals, mask, times = mtg.random_vertices_batch(N, D, 6, 16, [-5.0] * D, [5.0] * D, seed0=31,
                                                  max_derivative=N // 2 - 1)
    out = mtg.host_solve_linear_batch(N, r, vals, mask, times, status=True)
    assert np.all(out["status"] == 0)
    assert check_path(vals, mask, times, out["coeffs"], N, relative=True) < 1e-7
    if N <= 10:
        ref = O.solve_linear_batch(N, r, vals, mask.astype(np.uint32), times)
        assert scale_normalised_error(out["coeffs"], ref, times) <= ORACLE_TOL_N10
    else:
        # N = 12: the FP64 reference algorithm itself is 1e-4 from truth here (r = 0: 1.6e-4 .. 5.6e-4
        # on these problems), so the gate is 60-digit truth
        import os
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
        from make_golden import truth_solve
        for b in range(3):
            tr = truth_solve(N, r, vals[b], mask[b], times[b])[0]
            assert scale_normalised_error(out["coeffs"][b:b + 1], tr[None], times[b:b + 1]) <= TRUTH_TOL


def test_status_bits():
    vals, mask, times = mtg.random_vertices_path_batch(10, 3, 10, 6, seed0=4)
    times = times.copy()
    times[1, 3] = 0.0
    times[2, 0] = -1.0
    times[3, 5] = np.nan
    times[4, :] = 1e200  # T^k overflows: the pivots of R_pp are not finite (MTG_TRAJ_NOT_SPD)
    out = mtg.host_solve_linear_batch(10, 4, vals, mask, times, status=True)
    assert out["status"][0] == 0 and out["status"][5] == 0
    assert all(out["status"][i] & nat.MTG_TRAJ_BAD_TIME for i in (1, 2, 3))
    assert out["status"][4] & nat.MTG_TRAJ_NOT_SPD
    # 0 < T < DBL_EPSILON is a valid time for the reference's CHECK (lin_impl:287) but its A(T) is
    # singular there (baseCoeffsWithTime keeps only the t = 0 entry, polynomial.h:225): NOT_SPD
    t2 = times[:1].copy()
    t2[0, 4] = 1e-17
    tiny = mtg.host_solve_linear_batch(10, 4, vals[:1], mask[:1], t2, status=True)["status"][0]
    assert tiny & nat.MTG_TRAJ_NOT_SPD and not tiny & nat.MTG_TRAJ_BAD_TIME, tiny
    # orders > N/2-1 are dropped with a warning (lin_impl:74-95): same result as without them
    v8, m8, t8 = mtg.random_vertices_path_batch(8, 3, 6, 8)
    a = mtg.host_solve_linear_batch(8, 3, v8, m8, t8, status=True)
    b = mtg.host_solve_linear_batch(8, 3, v8, m8 & 0x0F, t8, status=True)
    assert np.all(a["status"] == nat.MTG_TRAJ_WARN_DROPPED) and np.all(b["status"] == 0)
    np.testing.assert_array_equal(a["coeffs"], b["coeffs"])
    with pytest.raises(nat.MTGError) as e:
        mtg.host_solve_linear_batch(10, 5, vals, mask, times)
    assert e.value.code == nat.MTG_ERR_BAD_DERIVATIVE


def test_free_values_ignored_and_threads_bitwise():
    vals, mask, times = mtg.random_vertices_path_batch(10, 3, 10, 300, seed0=8)
    a = mtg.host_solve_linear_batch(10, 4, vals, mask, times, cost=True)
    v2 = vals.copy()
    for k in range(5):
        v2[:, :, k, :][((mask >> k) & 1) == 0] = np.nan
    b = mtg.host_solve_linear_batch(10, 4, v2, mask, times, cost=True, threads=4)
    np.testing.assert_array_equal(a["coeffs"], b["coeffs"])
    np.testing.assert_array_equal(a["cost"], b["cost"])


def test_segment_matrices():
    """mtg_host_segment_matrices: A is the reference's setupMappingMatrix, A^-1 inverts it, Q is
    computeQuadraticCostJacobian, H = A^-T Q A^-1 (the oracle's FP64 restatements)."""
    import ctypes
    O = _oracle()
    lib = nat.load()
    for N, r in ((10, 4), (12, 3), (6, 0)):
        for T in (0.013, 1.0, 3.7, 41.0):
            A, Ai, Q, H = (np.zeros((N, N)) for _ in range(4))
            assert lib.mtg_host_segment_matrices(N, r, T, A.ctypes.data, Ai.ctypes.data, Q.ctypes.data,
                                                 H.ctypes.data) == 0
            np.testing.assert_array_equal(A, O.setup_mapping_matrix(N, T))
            np.testing.assert_allclose(Q, O.quadratic_cost_jacobian(N, r, T), rtol=1e-15, atol=0)
            Ai_ref = O.invert_mapping_matrix(A)
            # (the FP64 Schur inverse of the reference path loses up to ~2e-11 at N = 12, T = 0.013)
            assert np.max(np.abs(Ai - Ai_ref) / np.maximum(np.abs(Ai_ref), 1e-300)) < 1e-9
            H_ref = Ai_ref.T @ Q @ Ai_ref
            scale = np.sqrt(np.outer(np.abs(np.diag(H_ref)), np.abs(np.diag(H_ref)))) + 1e-300
            # forming A^-T Q A^-1 in FP64 (the reference path) costs digits at N = 12: 1.1e-7 at
            # T = 0.013; the exact table is the accurate side
            assert np.max(np.abs(H - H_ref) / scale) < (1e-8 if N <= 10 else 1e-6)
    assert lib.mtg_host_segment_matrices(10, 4, 0.0, None, None, None, None) == nat.MTG_ERR_INVALID_ARGUMENT
    assert lib.mtg_host_segment_matrices(10, 5, 1.0, None, None, None, None) == nat.MTG_ERR_BAD_DERIVATIVE
    del ctypes


def test_shard_range_partitions_the_batch():
    """mtg_shard_range: shard g of G is [g ceil(B/G), min(B, (g+1) ceil(B/G))) -- contiguous, disjoint,
    covering the batch; host solves of the shards concatenate bit-equal to one solve."""
    for B in (0, 1, 7, 37, 1000, 125001):
        for G in (1, 2, 3, 8):
            ranges = [mtg.shard_range(B, G, g) for g in range(G)]
            assert ranges[0][0] == 0 and ranges[-1][1] == B
            for (b0, b1), (c0, c1) in zip(ranges, ranges[1:]):
                assert b1 == c0 and b0 <= b1
            per = -(-B // G)
            assert all(b1 - b0 <= per for b0, b1 in ranges)
    with pytest.raises(nat.MTGError):
        mtg.shard_range(10, 2, 2)
    vals, mask, times = mtg.random_vertices_path_batch(10, 3, 10, 29, seed0=5)
    whole = mtg.host_solve_linear_batch(10, 4, vals, mask, times, free=True, cost=True, status=True)
    parts = [mtg.host_solve_linear_batch(10, 4, vals[b0:b1], mask[b0:b1], times[b0:b1], free=True, cost=True,
                                         status=True) for b0, b1 in (mtg.shard_range(29, 3, g) for g in range(3))]
    for k in ("coeffs", "free", "cost", "status"):
        np.testing.assert_array_equal(np.concatenate([p[k] for p in parts]), whole[k])


@pytest.mark.parametrize("derivative,dims", [(1, None), (2, None), (1, [1]), (3, [0, 2])])
def test_host_min_max_magnitude_vs_oracle(derivative, dims):
    """mtg_host_min_max_magnitude_batch (the drop-in's Trajectory::computeMinMaxMagnitude on the CPU)
    against the oracle (src/trajectory.cpp:181-218; numpy companion-matrix roots with the reference's
    |imag| <= eps filter)."""
    from oracle import pyoracle as O
    N, r, K, B = 10, 4, 10, 24
    vals, mask, times = mtg.random_vertices_path_batch(N, 3, K, B, seed0=1200)
    coeffs = mtg.host_solve_linear_batch(N, r, vals, mask, times)["coeffs"]
    mn, mx = mtg.host_min_max_magnitude_batch(coeffs, times, derivative, dims, threads=2)
    for b in range(B):
        rmn, rmx = O.min_max_magnitude(N, coeffs[b], times[b], derivative, dims)
        for got, ref in ((mx[b], rmx), (mn[b], rmn)):
            scale = max(abs(rmx[1]), 1e-300)
            assert abs(got["value"] - ref[1]) <= 1e-9 * scale, (b, got, ref)
            if got["segment"] == ref[2]:
                assert abs(got["time"] - ref[0]) <= 1e-6 * times[b, ref[2]] or abs(got["value"] - ref[1]) <= 1e-12 * scale


def test_host_solve_bitwise_fixture():
    """The host solve against its own earlier full-layout sweep, bit for bit: round 4
    restricted the forward and backward sweeps to each vertex's free derivatives, claimed bit-identical
    because the pinned rows and columns only added exact zeros.  tests/golden/make_host_fixture.py
    built the pre-change mtg_host_solve.cpp (commit 46c85dc) and recorded its coefficients, free
    values, n_free, cost and status on fully pinned / fully free vertices, free end derivatives, random
    pins and free positions, for 7 shapes."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "host_solve_bitwise.npz"))
    keys = sorted({k.split("__")[0] for k in g.files if "__" in k})
    assert len(keys) == 7
    for key in keys:
        N, D, K, r = (int(x[1:]) for x in key.split("_"))
        vals, mask, times = g[key + "__values"], g[key + "__mask"], g[key + "__times"]
        out = mtg.host_solve_linear_batch(N, r, vals, mask, times, free=True, n_free=True, cost=True, status=True)
        nf = g[key + "__n_free"]
        np.testing.assert_array_equal(out["coeffs"], g[key + "__coeffs"], err_msg=key)
        np.testing.assert_array_equal(out["n_free"], nf, err_msg=key)
        for b in range(len(nf)):
            np.testing.assert_array_equal(out["free"][b, :, :nf[b]], g[key + "__free"][b, :, :nf[b]], err_msg=key)
        np.testing.assert_array_equal(out["cost"], g[key + "__cost"], err_msg=key)
        np.testing.assert_array_equal(out["status"], g[key + "__status"], err_msg=key)


def test_host_solve_config4_truth_sample():
    """The config-4 truth sample (tests/golden/make_config4_truth.py: 256 trajectories of the full-size
    batch, 60-digit truth): the fixture's inputs still come out of the generator (SHA-256), and the host
    solve of the sample is within 1e-9 of truth (5.8e-11 when the fixture was made) -- the CPU half of
    the GPU test test_config4_full_size_truth_sample."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    import make_config4_truth as m
    g = np.load(os.path.join(here, "golden", "config4_truth_sample.npz"))
    vals, mask, times = m.batch()
    idx = g["index"]
    assert np.array_equal(idx, m.sample_index())
    assert m.inputs_digest(vals, mask, times, idx) == str(g["inputs_sha256"])
    h = mtg.host_solve_linear_batch(m.N, m.r, vals[idx], mask[idx], times[idx], status=True)
    assert np.all(h["status"] == 0)
    errs = [scale_normalised_error(h["coeffs"][i:i + 1], g["coeffs"][i:i + 1], times[idx][i:i + 1])
            for i in range(len(idx))]
    assert max(errs) <= 1e-9, max(errs)
