"""ctypes binding of libmav_trajectory_generation.so (the C ABI, include/mtg.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU
is visible, calls raise.  PyTorch is only used (in solver.py) as an optional
holder of device memory and streams.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmav_trajectory_generation.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "mtg.h")

MTG_OK = 0
MTG_ERR_INVALID_ARGUMENT = -1
MTG_ERR_UNSUPPORTED_N = -2
MTG_ERR_BAD_DERIVATIVE = -3
MTG_ERR_SIZE_MISMATCH = -4
MTG_ERR_HIP = -5
MTG_ERR_NO_DEVICE = -6
MTG_ERR_OUT_OF_MEMORY = -7
MTG_ERR_TOO_LARGE = -8

MTG_TRAJ_OK = 0
MTG_TRAJ_BAD_TIME = 1
MTG_TRAJ_NOT_SPD = 2
MTG_TRAJ_WARN_DROPPED = 256
MTG_TRAJ_ERROR_MASK = 255

MTG_FLAG_DEVICE_PTRS = 1
MTG_FLAG_ASYNC = 2
MTG_FLAG_SPLIT_KERNELS = 4
MTG_FLAG_GENERAL_KERNEL = 8
MTG_FLAG_DL_KERNEL = 64
MTG_FLAG_COLUMN_KERNEL = 128
MTG_DL_MIN_BATCH = 1

MTG_KERNEL_COLUMN = 2
MTG_KERNEL_GENERAL = 3
MTG_KERNEL_SPLIT = 4
MTG_KERNEL_DL = 6
MTG_KERNEL_DLX = 7
KERNEL_NAMES = {MTG_KERNEL_COLUMN: "solve_reg_kernel",
                MTG_KERNEL_GENERAL: "solve_fused_kernel", MTG_KERNEL_SPLIT: "assemble+block_cholesky",
                MTG_KERNEL_DL: "solve_dl_kernel", MTG_KERNEL_DLX: "solve_dlx_kernel"}

_c_dp = ctypes.c_void_p  # every array argument is passed as a raw address

_SIGNATURES = {
    "mtg_abi_version": (ctypes.c_int, []),
    "mtg_solve_kernel": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint]),
    "mtg_solve_kernel_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                              ctypes.c_uint]),
    "mtg_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "mtg_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "mtg_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "mtg_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "mtg_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "mtg_set_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "mtg_reset_stream": (ctypes.c_int, [ctypes.c_void_p]),
    "mtg_get_stream": (ctypes.c_void_p, [ctypes.c_void_p]),
    "mtg_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "mtg_solve_linear_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int64, _c_dp, _c_dp, _c_dp, _c_dp,
                                              _c_dp, _c_dp, _c_dp, _c_dp, ctypes.c_uint]),
    "mtg_shard_range": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64),
                                       ctypes.POINTER(ctypes.c_int64)]),
    "mtg_solve_linear_batch_multi": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_int, ctypes.c_int, ctypes.c_int64, _c_dp, _c_dp, _c_dp,
                                                    _c_dp, _c_dp, _c_dp, _c_dp, _c_dp, ctypes.c_uint]),
    "mtg_debug_fail_next_solve": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mtg_evaluate_range_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int64, _c_dp, _c_dp, ctypes.c_double, ctypes.c_double,
                                                ctypes.c_double, ctypes.c_int, _c_dp, _c_dp, _c_dp, _c_dp,
                                                ctypes.c_uint]),
    "mtg_evaluate_range_batch_full": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     ctypes.c_int64, _c_dp, _c_dp, ctypes.c_double, ctypes.c_double,
                                                     ctypes.c_double, ctypes.c_int, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp,
                                                     ctypes.c_int64, ctypes.c_uint]),
    "mtg_time_sweep_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int64, _c_dp, _c_dp, _c_dp, ctypes.c_int,
                                            _c_dp, _c_dp, _c_dp, ctypes.c_uint]),
    "mtg_cost_at_times_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int64, _c_dp, _c_dp, _c_dp, ctypes.c_int,
                                               _c_dp, _c_dp, _c_dp, ctypes.c_uint]),
    "mtg_time_jacobian_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int64, _c_dp, _c_dp, ctypes.c_int, _c_dp,
                                               ctypes.c_double, _c_dp, _c_dp, ctypes.c_uint]),
    "mtg_coefficients_from_vertices_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                            ctypes.c_int64, _c_dp, _c_dp, _c_dp, ctypes.c_uint]),
    "mtg_vertex_derivatives_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_int64, _c_dp, _c_dp, _c_dp, ctypes.c_uint]),
    "mtg_min_max_magnitude_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_int64, _c_dp, _c_dp, ctypes.c_int, ctypes.c_uint32,
                                                   _c_dp, _c_dp, ctypes.c_uint]),
    "mtg_last_kernel_ms": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]),
    "mtg_enable_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mtg_kernel_times": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_int)]),
    "mtg_host_solve_linear_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_int64, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp,
                                                   _c_dp, _c_dp, ctypes.c_int]),
    "mtg_host_default_threads": (ctypes.c_int, []),
    "mtg_host_min_max_magnitude_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                                        _c_dp, _c_dp, ctypes.c_int, ctypes.c_uint32, _c_dp, _c_dp,
                                                        ctypes.c_int]),
    "mtg_host_estimate_segment_times": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _c_dp, ctypes.c_double,
                                                       ctypes.c_double, ctypes.c_double, _c_dp]),
    "mtg_host_segment_matrices": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_double, _c_dp, _c_dp,
                                                 _c_dp, _c_dp]),
    "mtg_host_coefficients_from_vertices_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                                 ctypes.c_int64, _c_dp, _c_dp, _c_dp,
                                                                 ctypes.c_int]),
    "mtg_host_random_vertices_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                      _c_dp, _c_dp, ctypes.c_uint32, ctypes.c_int64,
                                                      ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                                      _c_dp, _c_dp, _c_dp, ctypes.c_int]),
    "mtg_host_random_vertices_path_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                           ctypes.c_double, ctypes.c_int, ctypes.c_uint32,
                                                           ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                                           ctypes.c_double, _c_dp, _c_dp, _c_dp,
                                                           ctypes.c_int]),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lib = None


class MTGError(RuntimeError):
    def __init__(self, code, message):
        super().__init__("%s (code %d)" % (message, code))
        self.code = code


def hip_runtimes_mapped():
    """Paths of the libamdhip64 images mapped into this process (Linux)."""
    found = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1]
                if "libamdhip64.so" in os.path.basename(p):
                    found.add(os.path.realpath(p))
    except OSError:
        pass
    return sorted(found)


def _share_torch_runtime():
    """PyTorch-ROCm wheels bundle their own libamdhip64 (soname libamdhip64.so.7, the
    same as /opt/rocm's).  Loading torch first makes the dynamic linker bind the library's
    libamdhip64.so.7 dependency to torch's already-loaded copy, so the process has ONE
    HIP runtime: torch stream handles and allocations are then valid in the library.  Loading
    the library first would map /opt/rocm's runtime and torch would later map a second one,
    whose streams/devices the library cannot see.  Set MTG_NO_TORCH=1 to skip (torch-free use)."""
    if os.environ.get("MTG_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load(path=None):
    """Load the library; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("MTG_LIBRARY", LIB_PATH)
    if not os.path.exists(p):
        raise MTGError(MTG_ERR_NO_DEVICE, "libmav_trajectory_generation.so not found at %s: run __graft_entry__.build()" % p)
    _share_torch_runtime()
    lib = ctypes.CDLL(p)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def status_string(code):
    return load().mtg_status_string(code).decode()


def check(code, ctx=None):
    if code != MTG_OK:
        msg = status_string(code)
        if ctx is not None:
            detail = load().mtg_last_error(ctx)
            if detail:
                msg += ": " + detail.decode()
        raise MTGError(code, msg)
    return code


def solve_kernel(N, D, K, r, flags=0, B=None):
    """Name of the solve kernel mtg_solve_linear_batch runs for this shape (mtg_solve_kernel), or for a
    batch of B trajectories (mtg_solve_kernel_batch: the default depends on B)."""
    lib = load()
    code = lib.mtg_solve_kernel(N, D, K, r, flags) if B is None else lib.mtg_solve_kernel_batch(N, D, K, r, B, flags)
    if code < 0:
        raise MTGError(code, status_string(code))
    return KERNEL_NAMES[code]


def device_count():
    n = ctypes.c_int(0)
    rc = load().mtg_device_count(ctypes.byref(n))
    return n.value if rc == MTG_OK else 0
