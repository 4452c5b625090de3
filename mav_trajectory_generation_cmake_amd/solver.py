"""Batched solver API over the C ABI (libmav_trajectory_generation.so).

Arrays may be numpy arrays (host; the library stages them through HBM) or
torch CUDA tensors (device-resident; launched on torch's current stream so
torch.cuda.Event timing and stream ordering work).  There is no CPU path.

Layouts follow include/mtg.h:
  values [B][K+1][N/2][D] float64, mask [B][K+1] uint8, times [B][K] float64
  coeffs [B][K][D][N], free [B][D][(K+1)*N/2], n_free [B], cost [B], status [B]
"""
import ctypes

import numpy as np

from . import _native as nat


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _addr(x):
    if x is None:
        return None
    if _is_torch(x):
        return x.data_ptr()
    return x.ctypes.data


# struct mtg_extremum (include/mtg.h)
EXTREMUM_DTYPE = np.dtype([("time", "<f8"), ("value", "<f8"), ("segment", "<i4"), ("reserved", "<i4")])


class Context:
    """Owns one mtg_ctx (a HIP stream + staging buffers on one device)."""

    def __init__(self, device=0):
        self._lib = nat.load()
        h = ctypes.c_void_p()
        nat.check(self._lib.mtg_create(device, ctypes.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            self._lib.mtg_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_stream(self, stream_handle):
        """Launch on this hipStream_t (an int, e.g. torch.cuda.current_stream().cuda_stream);
        0 / None is the HIP null stream (torch's default stream)."""
        nat.check(self._lib.mtg_set_stream(self.handle, stream_handle or None), self.handle)

    def reset_stream(self):
        """Launch on the context's own stream again."""
        nat.check(self._lib.mtg_reset_stream(self.handle), self.handle)

    def synchronize(self):
        nat.check(self._lib.mtg_synchronize(self.handle), self.handle)

    def last_kernel_ms(self):
        ms = ctypes.c_float(0)
        nat.check(self._lib.mtg_last_kernel_ms(self.handle, ctypes.byref(ms)), self.handle)
        return ms.value

    def enable_timing(self, ring):
        """Record a HIP event pair around each of the last `ring` kernel launches."""
        nat.check(self._lib.mtg_enable_timing(self.handle, ring), self.handle)

    def kernel_times_ms(self, n):
        """Durations (ms) of up to n most recent launches, oldest first (synchronizes)."""
        buf = (ctypes.c_float * max(n, 1))()
        got = ctypes.c_int(0)
        nat.check(self._lib.mtg_kernel_times(self.handle, buf, n, ctypes.byref(got)), self.handle)
        return np.array(buf[:got.value], dtype=np.float64)

    def solve_call(self, N, r, values, mask, times, coeffs, free=None, n_free=None, cost=None, status=None,
                   split=False, general=False, dl=False, column=False):
        """A zero-argument callable that launches one device-pointer solve asynchronously on the
        current stream with the arguments bound once (the bench's step; minimal host overhead)."""
        import torch
        B, V, h, D = values.shape
        K = V - 1
        self.set_stream(torch.cuda.current_stream(values.device).cuda_stream)
        flags = nat.MTG_FLAG_DEVICE_PTRS | nat.MTG_FLAG_ASYNC | (nat.MTG_FLAG_SPLIT_KERNELS if split else 0)
        flags |= nat.MTG_FLAG_GENERAL_KERNEL if general else 0
        flags |= nat.MTG_FLAG_DL_KERNEL if dl else 0
        flags |= nat.MTG_FLAG_COLUMN_KERNEL if column else 0
        fn = self._lib.mtg_solve_linear_batch
        args = (self.handle, N, D, K, r, B, _addr(values), _addr(mask), _addr(times), _addr(coeffs), _addr(free),
                _addr(n_free), _addr(cost), _addr(status), flags)
        handle = self.handle

        def call():
            rc = fn(*args)
            if rc:
                nat.check(rc, handle)
        return call

    def cost_call(self, N, r, vertex_values, times, scales, cost):
        """Zero-argument callable: one asynchronous device-pointer mtg_cost_at_times_batch launch on
        torch's current stream (the config-5 bench step)."""
        import torch
        B, V, h, D = vertex_values.shape
        C = scales.shape[0]
        self.set_stream(torch.cuda.current_stream(vertex_values.device).cuda_stream)
        fn = self._lib.mtg_cost_at_times_batch
        args = (self.handle, N, D, V - 1, r, B, _addr(vertex_values), None, _addr(times), C, _addr(scales),
                _addr(cost), None, nat.MTG_FLAG_DEVICE_PTRS | nat.MTG_FLAG_ASYNC)
        handle = self.handle

        def call():
            rc = fn(*args)
            if rc:
                nat.check(rc, handle)
        return call

    def jacobian_call(self, N, r, vertex_values, times, scales, cost, jac, increment_time=0.0):
        """Zero-argument callable: one asynchronous device-pointer mtg_time_jacobian_batch launch on
        torch's current stream (the config-5 bench step: cost sweep + time Jacobian, matrix cores)."""
        import torch
        B, V, h, D = vertex_values.shape
        C = scales.shape[0]
        self.set_stream(torch.cuda.current_stream(vertex_values.device).cuda_stream)
        fn = self._lib.mtg_time_jacobian_batch
        args = (self.handle, N, D, V - 1, r, B, _addr(vertex_values), _addr(times), C, _addr(scales),
                float(increment_time), _addr(cost), _addr(jac), nat.MTG_FLAG_DEVICE_PTRS | nat.MTG_FLAG_ASYNC)
        handle = self.handle

        def call():
            rc = fn(*args)
            if rc:
                nat.check(rc, handle)
        return call

    # ------------------------------------------------------------------ solve
    def solve_linear_batch(self, N, r, values, mask, times, coeffs=None, free=None, n_free=None,
                           cost=None, status=None, split=False, asynchronous=False, general=False, dl=False,
                           column=False):
        """Solve a batch; returns dict of outputs (allocates those not given).

        want-flags: pass arrays (or True to allocate) for free / n_free / cost / status."""
        dev = _is_torch(values) and values.is_cuda
        B, V, h, D = values.shape
        K = V - 1
        assert h == N // 2, "values must be [B][K+1][N/2][D]"
        assert tuple(mask.shape) == (B, V) and tuple(times.shape) == (B, K)
        out = {}

        def alloc(name, arr, shape, dtype):
            if arr is None or arr is False:
                return None
            if arr is True:
                if dev:
                    import torch
                    tdt = {np.float64: torch.float64, np.int32: torch.int32}[dtype]
                    arr = torch.empty(shape, dtype=tdt, device=values.device)
                else:
                    arr = np.empty(shape, dtype=dtype)
            out[name] = arr
            return arr

        coeffs = alloc("coeffs", True if coeffs is None else coeffs, (B, K, D, N), np.float64)
        free = alloc("free", free, (B, D, V * h), np.float64)
        n_free = alloc("n_free", n_free, (B,), np.int32)
        cost = alloc("cost", cost, (B,), np.float64)
        status = alloc("status", status, (B,), np.int32)
        flags = 0
        if dev:
            import torch
            flags |= nat.MTG_FLAG_DEVICE_PTRS
            self.set_stream(torch.cuda.current_stream(values.device).cuda_stream)
            if asynchronous:
                flags |= nat.MTG_FLAG_ASYNC
        else:
            values = np.ascontiguousarray(values, dtype=np.float64)
            mask = np.ascontiguousarray(mask, dtype=np.uint8)
            times = np.ascontiguousarray(times, dtype=np.float64)
            self.reset_stream()
        if split:
            flags |= nat.MTG_FLAG_SPLIT_KERNELS
        if general:
            flags |= nat.MTG_FLAG_GENERAL_KERNEL
        if dl:
            flags |= nat.MTG_FLAG_DL_KERNEL
        if column:
            flags |= nat.MTG_FLAG_COLUMN_KERNEL
        rc = self._lib.mtg_solve_linear_batch(self.handle, N, D, K, r, B, _addr(values), _addr(mask),
                                              _addr(times), _addr(coeffs), _addr(free), _addr(n_free),
                                              _addr(cost), _addr(status), flags)
        nat.check(rc, self.handle)
        return out

    def time_sweep_batch(self, N, r, values, mask, times, scales, cost=None, status=None,
                         asynchronous=False, split=False, dl=False, column=False, general=False):
        dev = _is_torch(values) and values.is_cuda
        B, V, h, D = values.shape
        K = V - 1
        C = len(scales)
        if dev:
            import torch
            cost = cost if cost is not None else torch.empty((B, C), dtype=torch.float64, device=values.device)
            flags = nat.MTG_FLAG_DEVICE_PTRS | (nat.MTG_FLAG_ASYNC if asynchronous else 0)
            self.set_stream(torch.cuda.current_stream(values.device).cuda_stream)
        else:
            values = np.ascontiguousarray(values, dtype=np.float64)
            mask = np.ascontiguousarray(mask, dtype=np.uint8)
            times = np.ascontiguousarray(times, dtype=np.float64)
            scales = np.ascontiguousarray(scales, dtype=np.float64)
            cost = cost if cost is not None else np.empty((B, C))
            flags = 0
            self.reset_stream()
        if split:
            flags |= nat.MTG_FLAG_SPLIT_KERNELS
        if dl:
            flags |= nat.MTG_FLAG_DL_KERNEL
        if column:
            flags |= nat.MTG_FLAG_COLUMN_KERNEL
        if general:
            flags |= nat.MTG_FLAG_GENERAL_KERNEL
        rc = self._lib.mtg_time_sweep_batch(self.handle, N, D, K, r, B, _addr(values), _addr(mask),
                                            _addr(times), C, _addr(scales), _addr(cost), _addr(status), flags)
        nat.check(rc, self.handle)
        return cost

    def cost_at_times_batch(self, N, r, vertex_values, times, scales, mask=None, grad=False):
        """getCostAndGradientDerivative at candidate times (include/mtg.h mtg_cost_at_times_batch):
        cost [B][C] = sum_dims d^T R(T_c) d, and with grad=True (needs mask) grad [B][C][D][V*h] =
        2 (R(T_c) d)_free in the reference's free order.  scales [C][K] multiply times [B][K]."""
        vertex_values = np.ascontiguousarray(vertex_values, dtype=np.float64)
        times = np.ascontiguousarray(times, dtype=np.float64)
        scales = np.ascontiguousarray(scales, dtype=np.float64)
        B, V, h, D = vertex_values.shape
        K = V - 1
        C = scales.shape[0]
        assert scales.shape == (C, K) and times.shape == (B, K)
        cost = np.empty((B, C))
        g = np.zeros((B, C, D, V * h)) if grad else None
        m = np.ascontiguousarray(mask, dtype=np.uint8) if mask is not None else None
        self.reset_stream()
        nat.check(self._lib.mtg_cost_at_times_batch(self.handle, N, D, K, r, B, _addr(vertex_values), _addr(m),
                                                    _addr(times), C, _addr(scales), _addr(cost), _addr(g), 0),
                  self.handle)
        return (cost, g) if grad else cost

    def time_jacobian_batch(self, N, r, vertex_values, times, scales, increment_time=0.0, jacobian=True):
        """Cost sweep + segment-time Jacobian on the matrix cores (include/mtg.h mtg_time_jacobian_batch):
        cost [B][C] = sum_dims d^T R(T_c) d and jac [B][C][K] = dJ/dT_i at T_c (exact for
        increment_time == 0, the reference's central difference otherwise)."""
        vertex_values = np.ascontiguousarray(vertex_values, dtype=np.float64)
        times = np.ascontiguousarray(times, dtype=np.float64)
        scales = np.ascontiguousarray(scales, dtype=np.float64)
        B, V, h, D = vertex_values.shape
        K = V - 1
        C = scales.shape[0]
        assert scales.shape == (C, K) and times.shape == (B, K)
        cost = np.empty((B, C))
        jac = np.empty((B, C, K)) if jacobian else None
        self.reset_stream()
        nat.check(self._lib.mtg_time_jacobian_batch(self.handle, N, D, K, r, B, _addr(vertex_values), _addr(times),
                                                    C, _addr(scales), float(increment_time), _addr(cost),
                                                    _addr(jac), 0), self.handle)
        return (cost, jac) if jacobian else cost

    def coefficients_from_vertices_batch(self, N, vertex_values, times):
        """setFreeConstraints + updateSegmentsFromCompactConstraints (include/mtg.h
        mtg_coefficients_from_vertices_batch): [B][V][h][D] all vertex derivatives -> [B][K][D][N]."""
        vertex_values = np.ascontiguousarray(vertex_values, dtype=np.float64)
        times = np.ascontiguousarray(times, dtype=np.float64)
        B, V, h, D = vertex_values.shape
        K = V - 1
        assert h == N // 2 and times.shape == (B, K)
        out = np.empty((B, K, D, N))
        self.reset_stream()
        nat.check(self._lib.mtg_coefficients_from_vertices_batch(self.handle, N, D, K, B, _addr(vertex_values),
                                                                 _addr(times), _addr(out), 0), self.handle)
        return out

    def vertex_derivatives_batch(self, coeffs, times):
        """M^+ A p (include/mtg.h mtg_vertex_derivatives_batch): [B][K][D][N] -> [B][V][h][D]."""
        coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
        times = np.ascontiguousarray(times, dtype=np.float64)
        B, K, D, N = coeffs.shape
        assert times.shape == (B, K)
        out = np.empty((B, K + 1, N // 2, D))
        self.reset_stream()
        nat.check(self._lib.mtg_vertex_derivatives_batch(self.handle, N, D, K, B, _addr(coeffs), _addr(times),
                                                         _addr(out), 0), self.handle)
        return out

    def set_free_constraints_batch(self, N, values, mask, times, free):
        """PolynomialOptimization::setFreeConstraints (polynomial_optimization_linear.h:185-186) for a
        batch: the fixed values stay, the free derivatives come from `free` [B][D][V*h] (reference
        order); returns the recomputed coefficients [B][K][D][N] (lin_impl:253-273)."""
        return self.coefficients_from_vertices_batch(N, full_vertex_values(values, mask, free, N), times)

    def initial_solution_without_position_constraints(self, N, r, values, mask, times):
        """PolynomialOptimizationNonLinear::computeInitialSolutionWithoutPositionConstraints
        (polynomial_optimization_nonlinear_impl.h:116-187) for a batch: solve, drop every position
        constraint except at the first and last vertex, and start the new free derivatives from the
        solved trajectory (M^+ A p).  Returns dict(mask, values, free [B][D][V*h], n_free, coeffs):
        the new problem (mask, values) and its free-constraint vector; re-solving it reproduces the
        same trajectory up to rounding."""
        values = np.ascontiguousarray(values, dtype=np.float64)
        B, V, h, D = values.shape
        sol = self.solve_linear_batch(N, r, values, mask, times)
        allv = self.vertex_derivatives_batch(sol["coeffs"], times)
        new_mask = np.array(mask, dtype=np.uint8, copy=True)
        new_mask[:, 1:V - 1] &= np.uint8(0xFE)  # vertices_[k].removeConstraint(POSITION), 0 < k < V-1
        fixed = ((new_mask[:, :, None] >> np.arange(h)[None, None, :]) & 1).astype(bool)  # [B][V][h]
        free = np.zeros((B, D, V * h))
        n_free = np.zeros(B, dtype=np.int32)
        for b in range(B):
            slots = np.flatnonzero(~fixed[b].reshape(-1))  # reference (vertex, derivative) order
            n_free[b] = len(slots)
            free[b, :, :len(slots)] = allv[b].reshape(-1, D)[slots].T
        return {"mask": new_mask, "values": values, "free": free, "n_free": n_free, "coeffs": sol["coeffs"]}

    def min_max_magnitude_batch(self, coeffs, times, derivative, dimensions=None):
        """Trajectory::computeMinMaxMagnitude (src/trajectory.cpp:181-218) for a batch (include/mtg.h
        mtg_min_max_magnitude_batch).  Returns (minimum, maximum), structured arrays [B] with fields
        time (segment-local), value, segment."""
        coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
        times = np.ascontiguousarray(times, dtype=np.float64)
        B, K, D, N = coeffs.shape
        mask = 0 if dimensions is None else int(sum(1 << int(d) for d in dimensions))
        mn = np.zeros(B, dtype=EXTREMUM_DTYPE)
        mx = np.zeros(B, dtype=EXTREMUM_DTYPE)
        self.reset_stream()
        nat.check(self._lib.mtg_min_max_magnitude_batch(self.handle, N, D, K, B, _addr(coeffs), _addr(times),
                                                        int(derivative), mask, _addr(mn), _addr(mx), 0),
                  self.handle)
        return mn, mx

    # ------------------------------------------------------- evaluateRange
    def evaluate_range_batch(self, coeffs, times, t_start, t_end, dt, derivative=0, want_times=True):
        """Host-array convenience wrapper: returns (samples [S][D], sample_times [S], counts [B], offsets [B])."""
        coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
        times = np.ascontiguousarray(times, dtype=np.float64)
        B, K, D, N = coeffs.shape
        counts = np.zeros(B, dtype=np.int64)
        self.reset_stream()
        nat.check(self._lib.mtg_evaluate_range_batch(self.handle, N, D, K, B, None, _addr(times), t_start, t_end,
                                                     dt, derivative, _addr(counts), None, None, None, 0),
                  self.handle)
        offsets = np.zeros(B, dtype=np.int64)
        if B > 1:
            offsets[1:] = np.cumsum(counts)[:-1]
        total = int(counts.sum())
        out = np.zeros((max(total, 1), D))
        st = np.zeros(max(total, 1)) if want_times else None
        nat.check(self._lib.mtg_evaluate_range_batch(self.handle, N, D, K, B, _addr(coeffs), _addr(times), t_start,
                                                     t_end, dt, derivative, _addr(counts), _addr(offsets),
                                                     _addr(out), _addr(st), 0), self.handle)
        return out[:total], (st[:total] if want_times else None), counts, offsets

    def evaluate_range_batch_full(self, coeffs, times, t_start, t_end, dt, derivative=0, want_times=True,
                                  capacity=None, asynchronous=False):
        """Trajectory::evaluateRange for the batch in one call (mtg_evaluate_range_batch_full): counts,
        offsets and samples computed on the device without a host round trip.  numpy arrays or torch
        CUDA tensors (then every output is a device tensor on torch's current stream).  capacity: rows
        of the sample buffer (default: evaluate_range_capacity, a safe bound); the call is retried
        once with the exact total if it was short.  Returns (samples [S][D], sample_times [S] or None,
        counts [B], offsets [B]); with asynchronous=True (device tensors only) the full-capacity
        buffers and the device total are returned instead of the trimmed views: (samples, times,
        counts, offsets, total)."""
        dev = _is_torch(coeffs) and coeffs.is_cuda
        B, K, D, N = coeffs.shape
        if capacity is None:
            capacity = evaluate_range_capacity(times, t_start, t_end, dt)
        for attempt in range(2):
            if dev:
                import torch
                kw = dict(device=coeffs.device)
                counts = torch.empty(B, dtype=torch.int64, **kw)
                offsets = torch.empty(B, dtype=torch.int64, **kw)
                total = torch.zeros(1, dtype=torch.int64, **kw)
                out = torch.empty((max(capacity, 1), D), dtype=torch.float64, **kw)
                st = torch.empty(max(capacity, 1), dtype=torch.float64, **kw) if want_times else None
                flags = nat.MTG_FLAG_DEVICE_PTRS | (nat.MTG_FLAG_ASYNC if asynchronous else 0)
                self.set_stream(torch.cuda.current_stream(coeffs.device).cuda_stream)
            else:
                coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
                times = np.ascontiguousarray(times, dtype=np.float64)
                counts = np.empty(B, dtype=np.int64)
                offsets = np.empty(B, dtype=np.int64)
                total = np.zeros(1, dtype=np.int64)
                out = np.empty((max(capacity, 1), D))
                st = np.empty(max(capacity, 1)) if want_times else None
                flags = 0
                self.reset_stream()
            rc = self._lib.mtg_evaluate_range_batch_full(self.handle, N, D, K, B, _addr(coeffs), _addr(times),
                                                         float(t_start), float(t_end), float(dt), int(derivative),
                                                         _addr(counts), _addr(offsets), _addr(total), _addr(out),
                                                         _addr(st), int(capacity), flags)
            if dev and asynchronous:
                nat.check(rc, self.handle)
                return out, st, counts, offsets, total
            if rc == nat.MTG_ERR_TOO_LARGE and attempt == 0:
                capacity = int(total[0])
                continue
            nat.check(rc, self.handle)
            break
        n = int(total[0])
        return out[:n], (st[:n] if want_times else None), counts, offsets


def evaluate_range_capacity(times, t_start, t_end, dt):
    """A safe sample capacity for evaluateRange over a batch (mtg_evaluate_range_batch_full): per
    trajectory the clock samples while the accumulated time (>= 0) is below t_end and the sample is
    inside the trajectory, so at most min(t_end, sum T) / dt + 2 samples; 1e-9 relative slack for the
    rounding of the accumulated clock."""
    if _is_torch(times):
        times = times.detach().cpu().numpy()
    span = np.minimum(np.asarray(times, dtype=np.float64).sum(axis=1), float(t_end))
    n = np.floor(np.maximum(span, 0.0) / float(dt) * (1.0 + 1e-9)) + 3
    return int(n.sum())


def full_vertex_values(values, mask, free, N):
    """All derivatives of every vertex [B][V][h][D]: the fixed values where the mask says fixed,
    the solved free values (free_out [B][D][V*h], reference order) elsewhere."""
    values = np.asarray(values, dtype=np.float64)
    B, V, h, D = values.shape
    fixed = ((np.asarray(mask)[:, :, None] >> np.arange(h)[None, None, :]) & 1).astype(bool)  # [B][V][h]
    out = np.where(fixed[..., None], values, 0.0)
    for b in range(B):
        slots = np.flatnonzero(~fixed[b].reshape(-1))  # (v, k) of free derivatives, reference order
        for d in range(D):
            out[b].reshape(-1, D)[slots, d] = free[b, d, :len(slots)]
    return out


_default_ctx = {}


def default_context(device=0):
    ctx = _default_ctx.get(device)
    if ctx is None:
        ctx = _default_ctx[device] = Context(device)
    return ctx


def solve_linear_batch(N, r, values, mask, times, device=0, **kw):
    return default_context(device).solve_linear_batch(N, r, values, mask, times, **kw)


def shard_range(batch, n_shards, shard):
    """[begin, end) of contiguous shard `shard` of `n_shards` (mtg_shard_range)."""
    b, e = ctypes.c_int64(0), ctypes.c_int64(0)
    nat.check(nat.load().mtg_shard_range(batch, n_shards, shard, ctypes.byref(b), ctypes.byref(e)))
    return b.value, e.value


def solve_linear_batch_multi(contexts, N, r, values, mask, times, free=False, n_free=False, cost=False,
                             status=False):
    """One batch over several contexts (normally one per device) in one call
    (mtg_solve_linear_batch_multi): contiguous shards, one host thread per context, host arrays in and
    out; bit-identical to one Context.solve_linear_batch over the whole batch."""
    lib = nat.load()
    values = np.ascontiguousarray(values, dtype=np.float64)
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    times = np.ascontiguousarray(times, dtype=np.float64)
    B, V, h, D = values.shape
    K = V - 1
    assert h == N // 2 and mask.shape == (B, V) and times.shape == (B, K)
    out = {"coeffs": np.empty((B, K, D, N))}
    if free:
        out["free"] = np.zeros((B, D, V * h))
    if n_free:
        out["n_free"] = np.empty((B,), np.int32)
    if cost:
        out["cost"] = np.empty((B,))
    if status:
        out["status"] = np.empty((B,), np.int32)
    handles = (ctypes.c_void_p * len(contexts))(*[c.handle for c in contexts])
    rc = lib.mtg_solve_linear_batch_multi(ctypes.cast(handles, ctypes.c_void_p), len(contexts), N, D, K, r, B,
                                          _addr(values), _addr(mask), _addr(times), _addr(out["coeffs"]),
                                          _addr(out.get("free")), _addr(out.get("n_free")), _addr(out.get("cost")),
                                          _addr(out.get("status")), 0)
    nat.check(rc, contexts[0].handle)
    return out


def host_min_max_magnitude_batch(coeffs, times, derivative, dimensions=None, threads=1):
    """The library's host path of Context.min_max_magnitude_batch (mtg_host_min_max_magnitude_batch):
    Trajectory::computeMinMaxMagnitude on the CPU, as the reference computes it (src/trajectory.cpp:181-218)."""
    lib = nat.load()
    coeffs = np.ascontiguousarray(coeffs, dtype=np.float64)
    times = np.ascontiguousarray(times, dtype=np.float64)
    B, K, D, N = coeffs.shape
    mask = 0 if dimensions is None else int(sum(1 << int(d) for d in dimensions))
    mn = np.zeros(B, dtype=EXTREMUM_DTYPE)
    mx = np.zeros(B, dtype=EXTREMUM_DTYPE)
    nat.check(lib.mtg_host_min_max_magnitude_batch(N, D, K, B, _addr(coeffs), _addr(times), int(derivative), mask,
                                                   _addr(mn), _addr(mx), threads))
    return mn, mx


def host_solve_linear_batch(N, r, values, mask, times, free=False, n_free=False, cost=False, status=False,
                            threads=1):
    """The library's host (CPU) solve path (mtg_host_solve_linear_batch): same algorithm and outputs as
    Context.solve_linear_batch, no GPU.  The drop-in PolynomialOptimization<N>::solveLinear uses it for
    single problems (BASELINE config 1)."""
    lib = nat.load()
    values = np.ascontiguousarray(values, dtype=np.float64)
    mask = np.ascontiguousarray(mask, dtype=np.uint8)
    times = np.ascontiguousarray(times, dtype=np.float64)
    B, V, h, D = values.shape
    K = V - 1
    assert h == N // 2, "values must be [B][K+1][N/2][D]"
    assert mask.shape == (B, V) and times.shape == (B, K)
    out = {"coeffs": np.empty((B, K, D, N))}
    if free:
        out["free"] = np.empty((B, D, V * h))
    if n_free:
        out["n_free"] = np.empty((B,), np.int32)
    if cost:
        out["cost"] = np.empty((B,))
    if status:
        out["status"] = np.empty((B,), np.int32)
    nat.check(lib.mtg_host_solve_linear_batch(N, D, K, r, B, _addr(values), _addr(mask), _addr(times),
                                              _addr(out["coeffs"]), _addr(out.get("free")),
                                              _addr(out.get("n_free")), _addr(out.get("cost")),
                                              _addr(out.get("status")), threads))
    return out


# ----------------------------------------------------------------- generators
def random_vertices_path_batch(N, D, K, batch, seed0=0, average_distance=5.0, max_derivative=4,
                               v_max=2.0, a_max=2.0, magic=6.5, threads=0):
    """The reference bench generator (src/polynomial_timing_evaluation.cpp:34-112), seeds seed0..seed0+B-1."""
    lib = nat.load()
    V, h = K + 1, N // 2
    values = np.zeros((batch, V, h, D))
    mask = np.zeros((batch, V), dtype=np.uint8)
    times = np.zeros((batch, K))
    nat.check(lib.mtg_host_random_vertices_path_batch(N, D, K, average_distance, max_derivative, seed0, batch,
                                                      v_max, a_max, magic, _addr(values), _addr(mask),
                                                      _addr(times), threads))
    return values, mask, times


def random_vertices_batch(N, D, K, batch, pos_min, pos_max, seed0=0, max_derivative=4, v_max=3.0, a_max=5.0,
                          magic=6.5, threads=0):
    """createRandomVertices + estimateSegmentTimes (src/vertex.cpp:27-79, :162-178)."""
    lib = nat.load()
    V, h = K + 1, N // 2
    pos_min = np.ascontiguousarray(pos_min, dtype=np.float64)
    pos_max = np.ascontiguousarray(pos_max, dtype=np.float64)
    assert len(pos_min) == D and len(pos_max) == D
    values = np.zeros((batch, V, h, D))
    mask = np.zeros((batch, V), dtype=np.uint8)
    times = np.zeros((batch, K))
    nat.check(lib.mtg_host_random_vertices_batch(N, D, K, max_derivative, _addr(pos_min), _addr(pos_max), seed0,
                                                 batch, v_max, a_max, magic, _addr(values), _addr(mask),
                                                 _addr(times), threads))
    return values, mask, times
