"""MI355X-native batched minimum-derivative polynomial trajectory optimizer.

Drop-in for the linear solve path of magrimm/mav_trajectory_generation_cmake
(PolynomialOptimization<N>::setupFromVertices + solveLinear, and
Trajectory::evaluateRange).  The compute path is hand-written HIP for gfx950
behind a C ABI (include/mtg.h, lib/libmav_trajectory_generation.so); this package is a thin Python
host layer over that ABI.  See DESIGN.md.
"""
from . import _native
from ._native import MTGError, device_count, load, solve_kernel
from .solver import (Context, default_context, full_vertex_values, host_min_max_magnitude_batch, host_solve_linear_batch, random_vertices_batch,
                     random_vertices_path_batch, shard_range, solve_linear_batch, solve_linear_batch_multi)

__all__ = ["MTGError", "Context", "default_context", "device_count", "full_vertex_values", "host_min_max_magnitude_batch",
           "host_solve_linear_batch",
           "load",
           "random_vertices_batch",
           "random_vertices_path_batch", "shard_range", "solve_kernel", "solve_linear_batch",
           "solve_linear_batch_multi", "_native"]
