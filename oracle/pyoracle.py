"""ctypes binding of the CPU restatement (oracle/mtg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

ORACLE_OK = 0
ORACLE_WARN_DROPPED = 1
ORACLE_ERR_ARG = -1
ORACLE_ERR_BAD_DERIVATIVE = -3
ORACLE_ERR_BAD_TIME = -4

_dp = ctypes.POINTER(ctypes.c_double)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_ip = ctypes.POINTER(ctypes.c_int)


class _Problem(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int), ("D", ctypes.c_int), ("K", ctypes.c_int), ("r", ctypes.c_int),
                ("nd", ctypes.c_int), ("values", _dp), ("mask", _u32p), ("times", _dp)]


class _Outputs(ctypes.Structure):
    _fields_ = [("coeffs", _dp), ("fixed", _dp), ("free_", _dp), ("col_of_row", _ip),
                ("ainv", _dp), ("amap", _dp), ("qmat", _dp), ("cost", _dp),
                ("counts", ctypes.c_int * 3)]


def build(build_dir=None, arch=None):
    """Compile liboracle.so (make); returns its path."""
    env = dict(os.environ)
    args = ["make", "-C", _HERE, "-s"]
    if build_dir:
        args.append("BUILD=%s" % build_dir)
    if arch:
        args.append("ARCH=%s" % arch)
    subprocess.check_call(args, env=env)
    return os.path.join(_HERE, build_dir or "_build", "liboracle.so")


def lib(path=None):
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    path = path or os.path.join(_HERE, "_build", "liboracle.so")
    if not os.path.exists(path):
        build()
    L = ctypes.CDLL(path)
    L.oracle_mt_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.oracle_mt_next.argtypes = [ctypes.c_void_p]
    L.oracle_mt_next.restype = ctypes.c_uint32
    L.oracle_uniform.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double]
    L.oracle_uniform.restype = ctypes.c_double
    L.oracle_base_coefficient.argtypes = [ctypes.c_int, ctypes.c_int]
    L.oracle_base_coefficient.restype = ctypes.c_double
    L.oracle_base_coeffs_with_time.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, _dp]
    L.oracle_poly_evaluate.argtypes = [ctypes.c_int, _dp, ctypes.c_double, ctypes.c_int]
    L.oracle_poly_evaluate.restype = ctypes.c_double
    L.oracle_create_random_vertices.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp,
                                                ctypes.c_uint32, ctypes.c_int, _dp, _u32p]
    L.oracle_create_random_vertices_path.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                                     ctypes.c_int, ctypes.c_uint32, ctypes.c_int, _dp, _u32p]
    L.oracle_estimate_segment_times.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp,
                                                ctypes.c_double, ctypes.c_double, ctypes.c_double, _dp]
    L.oracle_solve_linear.argtypes = [ctypes.POINTER(_Problem), ctypes.POINTER(_Outputs)]
    L.oracle_setup_mapping_matrix.argtypes = [ctypes.c_int, ctypes.c_double, _dp]
    L.oracle_invert_mapping_matrix.argtypes = [ctypes.c_int, _dp, _dp]
    L.oracle_quadratic_cost_jacobian.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, _dp]
    L.oracle_solve_linear_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int64, _dp, _u32p, _dp, _dp, _dp,
                                            ctypes.c_int]
    L.oracle_evaluate_range.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp,
                                        ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                        ctypes.c_int64, _dp, _dp]
    L.oracle_evaluate_range.restype = ctypes.c_int64
    L.oracle_cost_at_times_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int64, _dp, _dp, ctypes.c_int, _dp, _dp, ctypes.c_int]
    L.oracle_cost_time_jacobian_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                  ctypes.c_int, ctypes.c_int64, _dp, _dp, ctypes.c_int, _dp,
                                                  ctypes.c_double, _dp, _dp, ctypes.c_int]
    if path is None or _LIB is None:
        _LIB = L
    return L


def _p(a, t=_dp):
    return a.ctypes.data_as(t) if a is not None else None


class MT19937:
    """std::mt19937 restated (for golden checks)."""

    def __init__(self, seed):
        self._buf = ctypes.create_string_buffer(624 * 4 + 16)
        lib().oracle_mt_seed(self._buf, seed)

    def next(self):
        return lib().oracle_mt_next(self._buf)

    def uniform(self, a, b):
        return lib().oracle_uniform(self._buf, a, b)


def base_coefficient(n, i):
    return lib().oracle_base_coefficient(n, i)


def base_coeffs_with_time(N, d, t):
    out = np.zeros(N)
    lib().oracle_base_coeffs_with_time(N, d, t, _p(out))
    return out


def poly_evaluate(c, t, derivative=0):
    c = np.ascontiguousarray(c, dtype=np.float64)
    return lib().oracle_poly_evaluate(len(c), _p(c), t, derivative)


def create_random_vertices(max_derivative, K, pos_min, pos_max, seed, nd=None):
    pos_min = np.ascontiguousarray(pos_min, dtype=np.float64)
    pos_max = np.ascontiguousarray(pos_max, dtype=np.float64)
    D = len(pos_min)
    nd = nd or max(max_derivative + 1, 1)
    vals = np.zeros((K + 1, nd, D))
    mask = np.zeros(K + 1, dtype=np.uint32)
    rc = lib().oracle_create_random_vertices(max_derivative, K, D, _p(pos_min), _p(pos_max), seed, nd,
                                             _p(vals), _p(mask, _u32p))
    assert rc == 0
    return vals, mask


def create_random_vertices_path(D, K, average_distance, max_derivative, seed, nd=None):
    nd = nd or max(max_derivative + 1, 1)
    vals = np.zeros((K + 1, nd, D))
    mask = np.zeros(K + 1, dtype=np.uint32)
    rc = lib().oracle_create_random_vertices_path(D, K, average_distance, max_derivative, seed, nd,
                                                  _p(vals), _p(mask, _u32p))
    assert rc == 0
    return vals, mask


def estimate_segment_times(vals, v_max, a_max, magic=6.5):
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    V, nd, D = vals.shape
    t = np.zeros(V - 1)
    lib().oracle_estimate_segment_times(V - 1, D, nd, _p(vals), v_max, a_max, magic, _p(t))
    return t


def setup_mapping_matrix(N, T):
    A = np.zeros((N, N))
    lib().oracle_setup_mapping_matrix(N, T, _p(A))
    return A


def invert_mapping_matrix(A):
    A = np.ascontiguousarray(A, dtype=np.float64)
    out = np.zeros_like(A)
    lib().oracle_invert_mapping_matrix(A.shape[0], _p(A), _p(out))
    return out


def quadratic_cost_jacobian(N, r, T):
    Q = np.zeros((N, N))
    lib().oracle_quadratic_cost_jacobian(N, r, T, _p(Q))
    return Q


def solve_linear(N, r, vals, mask, times, want_matrices=False):
    """Run the restated setupFromVertices + solveLinear on one problem.

    vals [V][nd][D], mask [V] (bit k => derivative k fixed), times [K].
    Returns dict(rc, coeffs [K][D][N], fixed [D][nf], free [D][np], cost, counts, ...)."""
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    mask = np.ascontiguousarray(mask, dtype=np.uint32)
    times = np.ascontiguousarray(times, dtype=np.float64)
    V, nd, D = vals.shape
    K = V - 1
    h = N // 2
    n_all = (2 * V - 2) * h
    coeffs = np.zeros((K, D, N))
    fixed = np.zeros(D * V * h)
    free = np.zeros(D * V * h)
    cost = np.zeros(1)
    cor = np.zeros(n_all, dtype=np.int32)
    ainv = np.zeros((K, N, N)) if want_matrices else None
    amap = np.zeros((K, N, N)) if want_matrices else None
    qmat = np.zeros((K, N, N)) if want_matrices else None
    prob = _Problem(N, D, K, r, nd, _p(vals), _p(mask, _u32p), _p(times))
    out = _Outputs(_p(coeffs), _p(fixed), _p(free), _p(cor, _ip), _p(ainv), _p(amap), _p(qmat), _p(cost))
    rc = lib().oracle_solve_linear(ctypes.byref(prob), ctypes.byref(out))
    n_all_, nf, npf = out.counts[0], out.counts[1], out.counts[2]
    res = dict(rc=rc, coeffs=coeffs, cost=float(cost[0]), n_all=n_all_, n_fixed=nf, n_free=npf,
               fixed=fixed[:D * nf].reshape(D, nf), free=free[:D * npf].reshape(D, npf),
               col_of_row=cor)
    if want_matrices:
        res.update(ainv=ainv, amap=amap, qmat=qmat)
    return res


def solve_linear_batch(N, r, vals, mask, times, threads=0, want_cost=False):
    """vals [B][V][nd][D], mask [B][V] uint32, times [B][K]."""
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    mask = np.ascontiguousarray(mask, dtype=np.uint32)
    times = np.ascontiguousarray(times, dtype=np.float64)
    B, V, nd, D = vals.shape
    K = V - 1
    coeffs = np.zeros((B, K, D, N))
    cost = np.zeros(B) if want_cost else None
    rc = lib().oracle_solve_linear_batch(N, D, K, r, nd, B, _p(vals), _p(mask, _u32p), _p(times),
                                         _p(coeffs), _p(cost), threads)
    assert rc == 0, rc
    return (coeffs, cost) if want_cost else coeffs


def evaluate_range(coeffs, times, t_start, t_end, dt, derivative=0, max_samples=None):
    coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    K, D, N = coeffs.shape
    if max_samples is None:
        max_samples = int((t_end - t_start) / dt) + 16
    out = np.zeros((max_samples, D))
    st = np.zeros(max_samples)
    n = lib().oracle_evaluate_range(N, D, K, _p(coeffs), _p(times), t_start, t_end, dt, derivative,
                                    max_samples, _p(out), _p(st))
    m = min(n, max_samples)
    return out[:m], st[:m], n


def cost_at_times_batch(N, r, xfull, times, scales, threads=0):
    """getCostAndGradientDerivative's J at candidate times (oracle_cost_at_times_batch).
    xfull [B][V][nd][D], times [B][K], scales [C][K] -> J [B][C]."""
    xfull = np.ascontiguousarray(xfull, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    scales = np.ascontiguousarray(scales, dtype=np.float64)
    B, V, nd, D = xfull.shape
    C = scales.shape[0]
    J = np.zeros((B, C))
    rc = lib().oracle_cost_at_times_batch(N, D, V - 1, r, nd, B, _p(xfull), _p(times), C, _p(scales), _p(J), threads)
    assert rc == 0, rc
    return J


def cost_time_jacobian_batch(N, r, xfull, times, scales, increment_time=0.0, threads=0):
    """getCostAndGradientTime's J_d gradient at candidate times (oracle_cost_time_jacobian_batch).
    xfull [B][V][nd][D], times [B][K], scales [C][K] -> (J [B][C], G [B][C][K])."""
    xfull = np.ascontiguousarray(xfull, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    scales = np.ascontiguousarray(scales, dtype=np.float64)
    B, V, nd, D = xfull.shape
    C = scales.shape[0]
    J = np.empty((B, C))
    G = np.empty((B, C, V - 1))
    rc = lib().oracle_cost_time_jacobian_batch(N, D, V - 1, r, nd, B, _p(xfull), _p(times), C, _p(scales),
                                               float(increment_time), _p(J), _p(G), threads)
    assert rc == 0, rc
    return J, G


def vertex_derivatives(N, coeffs, times):
    """M^+ A p for one trajectory (polynomial_optimization_nonlinear_impl.h:162-180): A = blockdiag
    of setupMappingMatrix(T_i) (lin_impl:102-111), M the 0/1 reordering matrix in the reference's
    row order (segment i: vertex i derivatives 0..h-1, then vertex i+1; lin_impl:186-213) onto the
    unique (vertex, derivative) unknowns, M^+ = (M^T M)^-1 M^T.  coeffs [K][D][N] -> [V][h][D]."""
    coeffs = np.asarray(coeffs, dtype=np.float64)
    K, D, _ = coeffs.shape
    h, V = N // 2, K + 1
    M = np.zeros((K * N, V * h))
    for i in range(K):
        for s in range(N):
            M[i * N + s, (i + (s >= h)) * h + s % h] = 1.0
    Mp = np.linalg.pinv(M)
    out = np.zeros((V, h, D))
    for d in range(D):
        Ap = np.concatenate([setup_mapping_matrix(N, times[i]) @ coeffs[i, d] for i in range(K)])
        out[:, :, d] = (Mp @ Ap).reshape(V, h)
    return out


def coefficients_from_vertices(N, x, times):
    """updateSegmentsFromCompactConstraints (lin_impl:253-273) with every vertex derivative given:
    c_i = A(T_i)^-1 [x_i; x_{i+1}] with the reference's Schur inverse (lin_impl:133-169).
    x [V][h][D] -> coeffs [K][D][N]."""
    x = np.asarray(x, dtype=np.float64)
    V, h, D = x.shape
    K = V - 1
    out = np.zeros((K, D, N))
    for i in range(K):
        Ai = invert_mapping_matrix(setup_mapping_matrix(N, times[i]))
        for d in range(D):
            out[i, d] = Ai @ np.concatenate([x[i, :, d], x[i + 1, :, d]])
    return out


def _real_roots_in(poly_inc, t0, t1):
    """Real roots in [t0, t1] of a polynomial with INCREASING coefficients, selected as
    Polynomial::selectMinMaxCandidatesFromRoots does (src/polynomial.cpp:27-55: |imag| <= eps).
    The reference's root finder is Jenkins-Traub (src/rpoly.cpp); here LAPACK's companion-matrix
    eigenvalues (numpy.roots), which likewise return exactly-zero imaginary parts for roots it
    computes as real."""
    c = np.trim_zeros(np.asarray(poly_inc, dtype=np.float64), "b")
    if len(c) <= 1:
        return []
    r = np.roots(c[::-1])
    out = []
    for z in r:
        if abs(z.imag) > np.finfo(float).eps:
            continue
        if t0 <= z.real <= t1:
            out.append(float(z.real))
    return out


def min_max_magnitude(N, coeffs, times, derivative, dims=None):
    """Trajectory::computeMinMaxMagnitude (src/trajectory.cpp:181-218) for one trajectory.
    coeffs [K][D][N] -> ((t, value, segment) minimum, (t, value, segment) maximum)."""
    from math import factorial
    coeffs = np.asarray(coeffs, dtype=np.float64)
    K, D, _ = coeffs.shape
    dims = list(range(D)) if dims is None else list(dims)
    k = derivative

    def dcoef(c, m):  # getCoefficients(m): derivative coefficients, increasing powers
        return np.array([c[j + m] * factorial(j + m) / factorial(j) for j in range(N - m)])

    def mag(i, t):
        s = 0.0
        for d in dims:
            s += np.polyval(dcoef(coeffs[i, d], k)[::-1], t) ** 2
        return np.sqrt(s)

    mn, mx = (0.0, np.finfo(float).max, 0), (0.0, -np.finfo(float).max, 0)
    for i in range(K):
        T = float(times[i])
        if len(dims) > 1:  # segment.cpp:96-122
            nd, ndd = N - k, N - k - 1
            conv = np.zeros(nd + ndd - 1)
            for d in dims:
                conv += np.convolve(dcoef(coeffs[i, d], k)[:nd], dcoef(coeffs[i, d], k + 1)[:ndd])
            roots = _real_roots_in(conv, 0.0, T)
        else:  # one dimension: roots of p^(k+1) (segment.cpp:124-130)
            roots = _real_roots_in(dcoef(coeffs[i, dims[0]], k + 1), 0.0, T)
        cands = [0.0, T] + roots + [0.0, T]  # candidates, then start / end again (segment.cpp:172-193)
        smin, smax = (0.0, np.finfo(float).max), (0.0, -np.finfo(float).max)
        for t in cands:
            v = mag(i, t)
            if smax[1] < v:
                smax = (t, v)
            if v < smin[1]:
                smin = (t, v)
        if smin[1] < mn[1]:
            mn = (smin[0], smin[1], i)
        if smax[1] > mx[1]:
            mx = (smax[0], smax[1], i)
    return mn, mx
