/*
 * mtg.h -- C ABI of the MI355X batched minimum-derivative polynomial
 * optimizer (libmav_trajectory_generation.so).  Plain C types only: pointers, sizes, status codes.
 *
 * The reference (magrimm/mav_trajectory_generation_cmake) has no FFI; its
 * boundary is the C++ template class PolynomialOptimization<N>
 * (mav_trajectory_generation/include/mav_trajectory_generation/
 * polynomial_optimization_linear.h:45-269).  Each entry point below states
 * which reference interface it replaces.  The C++ drop-in headers at the
 * reference's include paths (include/mav_trajectory_generation/ headers, namespace
 * mav_trajectory_generation) are written on top of this ABI, and
 * INTEGRATION.md shows the bindings (C++, CMake, ctypes) a maintainer adds.
 *
 * Rules: the library never aborts and never throws; calls return MTG_OK or a
 * negative MTG_ERR_*.  All buffers are caller-owned and never retained after
 * a call returns (with MTG_FLAG_ASYNC: until the stream is synchronized).
 * One mtg_ctx serialises its calls; different contexts are thread-safe.
 *
 * Data layout (all FP64, row-major, B = batch, V = K + 1 vertices,
 * h = N / 2 derivatives 0..h-1 per vertex, D dimensions):
 *   values   [B][V][h][D]  value of derivative k at vertex v, dimension d
 *                          (read only where the derivative is fixed)
 *   fixed_mask [B][V]      uint8, bit k set => derivative k of vertex v is
 *                          fixed (Vertex::addConstraint, vertex.h:58-64);
 *                          bits >= h are dropped with a warning status, as
 *                          setupFromVertices does (lin_impl:74-95)
 *   times    [B][K]        segment times, must be > 0 (lin_impl:287)
 *   coeffs   [B][K][D][N]  polynomial coefficients, increasing powers
 *                          (polynomial_optimization_linear.h:42-44)
 *   free_out [B][D][V*h]   optional: getFreeConstraints() values
 *                          (polynomial_optimization_linear.h:180-184) in the
 *                          reference order (sorted by vertex, then derivative)
 *   n_free_out [B]         optional: getNumberFreeConstraints()
 *   cost_out [B]           optional: computeCost() = 0.5 sum c^T Q c
 *                          (lin_impl:114-130)
 *   status   [B]           optional: per-trajectory MTG_TRAJ_* bits
 * ("lin_impl" = .../impl/polynomial_optimization_linear_impl.h)
 */
#ifndef MTG_H_
#define MTG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTG_ABI_VERSION 1

/* Call-level return codes. */
#define MTG_OK 0
#define MTG_ERR_INVALID_ARGUMENT (-1)
#define MTG_ERR_UNSUPPORTED_N (-2)     /* N must be even, 2 <= N <= 12 (polynomial.h:46) */
#define MTG_ERR_BAD_DERIVATIVE (-3)    /* 0 <= r <= N/2-1 (lin_impl:50-55) */
#define MTG_ERR_SIZE_MISMATCH (-4)     /* K < 1, D < 1, B < 0 (lin_impl:66-67, :279-281) */
#define MTG_ERR_HIP (-5)               /* HIP runtime error, see mtg_last_error() */
#define MTG_ERR_NO_DEVICE (-6)
#define MTG_ERR_OUT_OF_MEMORY (-7)
#define MTG_ERR_TOO_LARGE (-8)         /* per-trajectory working set exceeds LDS */

/* Per-trajectory status bits (status[b]). */
#define MTG_TRAJ_OK 0
#define MTG_TRAJ_BAD_TIME 1            /* some T <= 0 or not finite (CHECK_GT lin_impl:287) */
#define MTG_TRAJ_NOT_SPD 2             /* non-positive pivot in R_pp (reference: undetected, lin_impl:355-368),
                                          or some 0 < T < DBL_EPSILON, where the reference's A(T) is
                                          singular (baseCoeffsWithTime, polynomial.h:225) */
#define MTG_TRAJ_WARN_DROPPED 256      /* constraint of order > N/2-1 ignored (LOG(WARNING) lin_impl:84-87) */
#define MTG_TRAJ_ERROR_MASK 255

/* Flags. */
#define MTG_FLAG_DEVICE_PTRS 1u        /* all array arguments are device pointers on the ctx device */
#define MTG_FLAG_ASYNC 2u              /* do not synchronize the stream before returning */
#define MTG_FLAG_SPLIT_KERNELS 4u      /* two-kernel path: assembly kernel + block-Cholesky kernel */
#define MTG_FLAG_GENERAL_KERNEL 8u     /* diagnostics: always use the general LDS-resident fused kernel
                                          (default: see mtg_solve_kernel) */
/* Deprecated (ABI 1 names kept so round-3 callers still compile): 16u and 32u selected the
 * lane-per-chain and interior-waypoint lane kernels, retired in round 4 (measured slower than the
 * default everywhere).  The bits are reserved and ignored: a call that sets them runs
 * the default kernel, and mtg_solve_kernel never returns MTG_KERNEL_LANE or MTG_KERNEL_IP. */
#define MTG_FLAG_LANE_KERNEL 16u       /* deprecated, ignored */
#define MTG_FLAG_IP_KERNEL 32u         /* deprecated, ignored */

#define MTG_FLAG_DL_KERNEL 64u         /* the dimension-lane kernel where it applies (N = 10 with K = 10,
                                          N = 12 with K = 20; D <= 4, r >= 1; one lane per (chain,
                                          dimension)).  The reference generators' pattern takes its pattern
                                          pass, any other mask with every position fixed its general-mask
                                          pass, and a trajectory with a free position the general fused
                                          kernel's block function inside it (with that kernel's bits):
                                          DESIGN.md 3.2c.  The default for those shapes at every batch size */
#define MTG_FLAG_COLUMN_KERNEL 128u    /* the register column kernel wherever it applies, also where the
                                          default for the batch size is the dimension-lane kernel (A/B) */
#define MTG_DL_MIN_BATCH 1             /* Deprecated (round 3: 2048; kept as 1 for callers that test it).
                                          Since round 4 the dimension-lane kernel is the
                                          default at every batch size where it applies, so a trajectory's
                                          result never depends on the size of the call or on the other
                                          trajectories in it (it was faster at every size) */

/* Solve kernels (mtg_solve_kernel): which one mtg_solve_linear_batch runs for a shape.  (1 and 5,
   MTG_KERNEL_LANE and MTG_KERNEL_IP, named the kernels retired in round 4: deprecated, never returned.) */
#define MTG_KERNEL_LANE 1              /* deprecated */
#define MTG_KERNEL_IP 5                /* deprecated */
#define MTG_KERNEL_COLUMN 2            /* default: register column kernel, a lane per column of G_v /
                                          per dimension, twisted (K <= 12, N = 12 up to K = 20) */
#define MTG_KERNEL_GENERAL 3           /* general LDS-resident fused kernel (any K) */
#define MTG_KERNEL_SPLIT 4             /* assembly kernel + block-Cholesky kernel */
#define MTG_KERNEL_DL 6                /* one lane per (chain, dimension) (MTG_FLAG_DL_KERNEL) */
#define MTG_KERNEL_DLX 7               /* the same for chains of other lengths (N = 10 / 12, D <= 4, r >= 1,
                                          where neither the DL nor the column kernel applies: e.g. the
                                          reference benchmark's K = 50 / 100), plus the general kernel's
                                          block function for trajectories whose interior vertices do not
                                          fix exactly their position */

typedef struct mtg_ctx mtg_ctx;

/* Version / diagnostics. */
int mtg_abi_version(void);
/* The solve kernel (MTG_KERNEL_*) mtg_solve_linear_batch runs for this shape and these flags, or a
   negative MTG_ERR_* for a shape it rejects.  No device work. */
int mtg_solve_kernel(int N, int D, int K, int derivative_to_optimize, unsigned flags);
/* The same for a batch of B trajectories (or trajectory x candidate pairs).  Since round 4 the answer
   does not depend on B (kept for round-3 callers). */
int mtg_solve_kernel_batch(int N, int D, int K, int derivative_to_optimize, int64_t B, unsigned flags);
const char* mtg_status_string(int code);
const char* mtg_last_error(mtg_ctx* ctx);

/* Devices and contexts.  A context owns a HIP stream on one device plus
 * staging buffers for host-pointer calls. */
int mtg_device_count(int* count);
int mtg_create(int device, mtg_ctx** out_ctx);
int mtg_destroy(mtg_ctx* ctx);
/* Launch on an external hipStream_t (e.g. torch's current stream).  NULL
 * selects the HIP null (default) stream; mtg_reset_stream restores the
 * context's own stream. */
int mtg_set_stream(mtg_ctx* ctx, void* hip_stream);
int mtg_reset_stream(mtg_ctx* ctx);
void* mtg_get_stream(mtg_ctx* ctx);
int mtg_synchronize(mtg_ctx* ctx);

/* Batched setupFromVertices + solveLinear.  Replaces, per trajectory,
 *   PolynomialOptimization<N>(D)                 lin_impl:33-44
 *   setupFromVertices(vertices, times, r)        lin_impl:47-99
 *     updateSegmentTimes                         lin_impl:276-295
 *     setupConstraintReorderingMatrix            lin_impl:172-250
 *   solveLinear()                                lin_impl:329-369
 *     constructR + SparseQR + per-dim solve      lin_impl:298-365
 *     updateSegmentsFromCompactConstraints       lin_impl:253-273
 *   getSegments / getFreeConstraints / computeCost.
 * One call solves B independent problems of identical shape (N, D, K, r);
 * masks and values may differ per trajectory. */
int mtg_solve_linear_batch(mtg_ctx* ctx, int N, int D, int K, int derivative_to_optimize,
                           int64_t batch, const double* values, const uint8_t* fixed_mask,
                           const double* times, double* coeffs, double* free_out,
                           int32_t* n_free_out, double* cost_out, int32_t* status,
                           unsigned flags);

/* Contiguous shard `shard` (0 <= shard < n_shards) of a batch of `batch` independent problems:
 * [*begin, *end) = [g ceil(B/G), min(B, (g+1) ceil(B/G))).  The partition that
 * mtg_solve_linear_batch_multi, bench.py's ranks and the Python layer use.  No device work. */
int mtg_shard_range(int64_t batch, int n_shards, int shard, int64_t* begin, int64_t* end);

/* mtg_solve_linear_batch over several contexts, normally one per device (mtg_create(g, ...)), in one
 * call: the batch is cut into n_ctxs contiguous shards (mtg_shard_range) and shard g is solved by
 * ctxs[g] on its own host thread (the calling thread takes shard 0), each with its own staging /
 * chunk pipeline, writing its disjoint slice of the outputs.  Trajectories are independent, so there
 * is no collective.  This replaces a caller's loop of single solves over a whole batch
 * (src/polynomial_timing_evaluation.cpp:119-126) with one call that uses every GPU of the node.
 * Host arrays only (MTG_FLAG_DEVICE_PTRS and MTG_FLAG_ASYNC are rejected: device arrays live on one
 * device); the call returns when every shard has landed.  Results are bit-identical to one
 * mtg_solve_linear_batch over the whole batch.  On failure the first failing shard's code is
 * returned and mtg_last_error(ctxs[0]) names the shard.  Distinct contexts run concurrently; a
 * context listed twice serialises its shards. */
int mtg_solve_linear_batch_multi(mtg_ctx* const* ctxs, int n_ctxs, int N, int D, int K, int derivative_to_optimize,
                                 int64_t batch, const double* values, const uint8_t* fixed_mask,
                                 const double* times, double* coeffs, double* free_out, int32_t* n_free_out,
                                 double* cost_out, int32_t* status, unsigned flags);

/* Diagnostics: the next mtg_solve_linear_batch on ctx (also as one shard of a multi-device solve)
 * returns `code` (a negative MTG_ERR_*) without touching any array, as a failing device would --
 * for testing how a caller or mtg_solve_linear_batch_multi propagates a shard's failure. */
int mtg_debug_fail_next_solve(mtg_ctx* ctx, int code);

/* Batched Trajectory::evaluateRange (src/trajectory.cpp:68-128) over solved
 * trajectories, with the reference's sequential time accumulation (acc += dt)
 * reproduced exactly.  coeffs [B][K][D][N], times [B][K].  Sample counts are
 * ragged: first call with out == NULL to get counts[B] (samples per
 * trajectory); then pass the same counts (read), offsets[B] (exclusive prefix
 * sum of counts, in samples) and out [sum(counts)][D] (+ optional
 * sample_times [sum]).
 * t_start/t_end/dt are shared by the whole batch; derivative selects the
 * derivative order evaluated (Polynomial::evaluate, polynomial.h:138-151). */
int mtg_evaluate_range_batch(mtg_ctx* ctx, int N, int D, int K, int64_t batch,
                             const double* coeffs, const double* times, double t_start,
                             double t_end, double dt, int derivative, int64_t* counts,
                             const int64_t* offsets, double* out, double* sample_times,
                             unsigned flags);

/* Batched Trajectory::evaluateRange in ONE call (the samples' total is not known in advance):
 * counts[B] (samples per trajectory), offsets[B] (exclusive prefix sum of counts, in samples),
 * *total (the sum) and the samples out [total][D] (+ sample_times [total], nullable) -- all computed
 * on the device with no host round trip between them (the clock kernel also counts and scans; the
 * sample kernel adds the block offsets).  `capacity` is the number of sample rows out (and
 * sample_times) can hold.  If *total exceeds it, no sample is written and the call returns
 * MTG_ERR_TOO_LARGE after counts, offsets and *total are filled (retry with capacity = *total); with
 * MTG_FLAG_DEVICE_PTRS | MTG_FLAG_ASYNC the caller checks *total itself.  A safe capacity per
 * trajectory is min(t_end, sum T_i) / dt + 2 (samples are taken while the accumulated time is below
 * t_end and inside the trajectory), summed over the batch, with a little slack for the rounding of
 * the accumulated clock.  With MTG_FLAG_DEVICE_PTRS every array (and total) is a device pointer;
 * otherwise all are host pointers (the call then reads the total back once to size its staging). */
int mtg_evaluate_range_batch_full(mtg_ctx* ctx, int N, int D, int K, int64_t batch, const double* coeffs,
                                  const double* times, double t_start, double t_end, double dt, int derivative,
                                  int64_t* counts, int64_t* offsets, int64_t* total, double* out,
                                  double* sample_times, int64_t capacity, unsigned flags);

/* Batched segment-time sweep (the nonlinear time-allocation objective,
 * polynomial_optimization_nonlinear_impl.h:765-832 via updateSegmentTimes +
 * solveLinear + computeCost): for each trajectory b and candidate c the
 * times are scale[c] * times[b][:] and the result is the optimal cost
 * J(b, c) (computeCost()).  cost_out [B][C]. */
int mtg_time_sweep_batch(mtg_ctx* ctx, int N, int D, int K, int derivative_to_optimize,
                         int64_t batch, const double* values, const uint8_t* fixed_mask,
                         const double* times, int n_candidates, const double* scales,
                         double* cost_out, int32_t* status, unsigned flags);

/* Cost (and gradient) of FIXED vertex derivatives at candidate segment times: the reference's
 * getCostAndGradientDerivative (polynomial_optimization_nonlinear_impl.h:1452-1520) evaluated at
 * perturbed times, as its numerical time gradient does (getCostAndGradientTime :2153-2238):
 *   J(b, c) = sum_dims d^T R(T_c) d   (no 1/2, unlike computeCost)
 *   grad(b, c, dim) = 2 (R(T_c) d)_free   (free derivatives in the reference (vertex, derivative)
 *                                          order; only with fixed_mask, entries >= n_free left 0)
 * with T_c[i] = times[b][i] * scales[c][i].  vertex_values [B][V][h][D] holds ALL derivatives of
 * every vertex (fixed values and the solved free ones, e.g. from free_out); fixed_mask [B][V] is
 * needed only for the gradient.  cost_out [B][C]; grad_out [B][C][D][V*h] (nullable). */
int mtg_cost_at_times_batch(mtg_ctx* ctx, int N, int D, int K, int derivative_to_optimize,
                            int64_t batch, const double* vertex_values, const uint8_t* fixed_mask,
                            const double* times, int n_candidates, const double* scales,
                            double* cost_out, double* grad_out, unsigned flags);

/* Segment-time sweep of the fixed-derivative cost with its time Jacobian (BASELINE config 5, the
 * matrix-core path).  Replaces, per trajectory b and candidate allocation c,
 *   updateSegmentTimes(T_c) + getCostAndGradientDerivative(NULL)      nl_impl:1452-1520
 * and the J_d part of getCostAndGradientTime's per-segment gradient    nl_impl:2153-2238
 * (dJd_dt; the collision, soft-constraint and w_* weighting terms are not part of this path):
 *   cost_out[b][c]      = sum_dims d^T R(T_c) d                 (as mtg_cost_at_times_batch)
 *   jac_out[b][c][i]    = dJ/dT_i at T_c                        (nullable)
 * with T_c[i] = times[b][i] * scales[c][i] and d = vertex_values[b] (ALL derivatives of every
 * vertex, fixed and solved free ones).  increment_time == 0 gives the exact derivative;
 * increment_time > 0 gives the reference's central difference
 *   (J(T_i + dt) - J(T_i - dt)) / (2 dt), both perturbed times 0.1 when T_i <= 0.1
 * (nl_impl:2180-2223; the reference default is increment_time = 0.1,
 * polynomial_optimization_nonlinear.h:67); NaN where T_i - dt <= 0 (the reference CHECK-fails).
 * Works for any n_candidates >= 1; per-call LDS limits the shape (MTG_ERR_TOO_LARGE). */
int mtg_time_jacobian_batch(mtg_ctx* ctx, int N, int D, int K, int derivative_to_optimize,
                            int64_t batch, const double* vertex_values, const double* times,
                            int n_candidates, const double* scales, double increment_time,
                            double* cost_out, double* jac_out, unsigned flags);

/* Coefficients from ALL vertex derivatives (fixed and free), nothing solved: per trajectory the
 * reference's setFreeConstraints (polynomial_optimization_linear.h:185-186) followed by
 * updateSegmentsFromCompactConstraints (lin_impl:253-273), c_i = A(T_i)^-1 [x_i; x_{i+1}].
 * vertex_values [B][V][h][D], times [B][K] (> 0) -> coeffs [B][K][D][N]. */
int mtg_coefficients_from_vertices_batch(mtg_ctx* ctx, int N, int D, int K, int64_t batch,
                                         const double* vertex_values, const double* times, double* coeffs,
                                         unsigned flags);

/* Vertex derivatives of solved trajectories: the reference's M^+ A p
 * (polynomial_optimization_nonlinear_impl.h:162-180, computeInitialSolutionWithoutPositionConstraints;
 * getA / getMpinv, polynomial_optimization_linear.h:209-214): derivative k < h of every segment end,
 * averaged over the two segment ends meeting at an interior vertex.
 * coeffs [B][K][D][N], times [B][K] -> vertex_values [B][V][h][D]. */
int mtg_vertex_derivatives_batch(mtg_ctx* ctx, int N, int D, int K, int64_t batch, const double* coeffs,
                                 const double* times, double* vertex_values, unsigned flags);

/* Extremum of a trajectory (the reference's Extremum, extremum.h): segment-local time, value and
 * segment index. */
typedef struct mtg_extremum {
  double time;
  double value;
  int32_t segment;
  int32_t reserved;
} mtg_extremum;

/* Minimum and maximum magnitude of derivative `derivative` (0 <= derivative <= N-2) over each
 * whole trajectory: Trajectory::computeMinMaxMagnitude (src/trajectory.cpp:181-218) with the
 * dimensions in dimension_mask (bit d = dimension d; 0 = all).  Per segment the candidates are
 * t = 0, t = T and the real roots in [0, T] of sum_d conv(p_d^(k), p_d^(k+1)) (one dimension: of
 * p^(k+1)), src/segment.cpp:82-196.  coeffs [B][K][D][N], times [B][K]; minimum / maximum [B]
 * (either may be NULL).  Roots are isolated on 256 samples per segment and refined to a few ulp
 * (the reference uses Jenkins-Traub, src/rpoly.cpp); see DESIGN.md. */
int mtg_min_max_magnitude_batch(mtg_ctx* ctx, int N, int D, int K, int64_t batch, const double* coeffs,
                                const double* times, int derivative, uint32_t dimension_mask,
                                mtg_extremum* minimum, mtg_extremum* maximum, unsigned flags);

/* Timing of the most recent kernel launch(es) of this context on its stream
 * (hipEvent pair around the solve kernel), in milliseconds. */
int mtg_last_kernel_ms(mtg_ctx* ctx, float* ms);
/* Keep a HIP event pair per launch for the last `ring` launches (ring >= 0;
 * the default is 1; 0 records no events).  Single-kernel calls carry the pair in
 * the kernel's dispatch packet.  mtg_kernel_times synchronizes on the newest event and
 * writes up to n durations (ms, oldest first) of the launches still in the
 * ring; *n_out receives the count. */
int mtg_enable_timing(mtg_ctx* ctx, int ring);
int mtg_kernel_times(mtg_ctx* ctx, float* ms, int n, int* n_out);

/* Host (CPU) path of mtg_solve_linear_batch, no context and no GPU needed: the same algorithm
 * as the HIP kernels (exact tables, symmetric pinning, block LDL^T Thomas), in scalar C++ on the
 * calling thread(s).  For one problem it is the lowest-latency path (a GPU round trip costs more
 * than the solve itself): the C++ drop-in PolynomialOptimization<N>::solveLinear uses it by
 * default (BASELINE config 1), replacing the reference's CPU solveLinear (lin_impl:329-369).
 * Same arrays and per-trajectory status as mtg_solve_linear_batch, all host pointers;
 * threads <= 0: mtg_host_default_threads(). */
int mtg_host_solve_linear_batch(int N, int D, int K, int derivative_to_optimize, int64_t batch,
                                const double* values, const uint8_t* fixed_mask, const double* times,
                                double* coeffs, double* free_out, int32_t* n_free_out, double* cost_out,
                                int32_t* status, int threads);

/* The worker count the host paths (mtg_host_*) use when called with threads <= 0: the CPUs this
 * process may run on -- its affinity mask, capped by the cgroup CPU quota -- not every CPU of the
 * machine.  (The reference's host code is single-threaded; there is no reference counterpart.) */
int mtg_host_default_threads(void);

/* Host (CPU) path of mtg_min_max_magnitude_batch, no context and no GPU needed: the same candidates,
 * root isolation and tie rules as the HIP kernel, on the calling thread(s).  The reference computes
 * Trajectory::computeMinMaxMagnitude on the CPU (src/trajectory.cpp:181-218); the C++ drop-in uses
 * this for its single trajectories unless ExecutionPolicy::kDevice.  All host pointers; threads <= 0:
 * mtg_host_default_threads(). */
int mtg_host_min_max_magnitude_batch(int N, int D, int K, int64_t batch, const double* coeffs, const double* times,
                                     int derivative, uint32_t dimension_mask, mtg_extremum* minimum,
                                     mtg_extremum* maximum, int threads);

/* ---- Host utilities (no GPU): the reference's synthetic-input generators,
 * bit-exact with libstdc++ <random>, packed straight into the ABI layout.
 * Trajectory b of a batch uses seed (seed0 + b).  values [B][V][h][D],
 * fixed_mask [B][V]; derivatives above N/2-1 set the WARN_DROPPED bit in the
 * returned mask (bit 7) and are otherwise ignored, as setupFromVertices does. */
/* createRandomVertices (src/vertex.cpp:27-79) + estimateSegmentTimes (:162-178) */
int mtg_host_random_vertices_batch(int N, int D, int K, int max_derivative, const double* pos_min,
                                   const double* pos_max, uint32_t seed0, int64_t batch,
                                   double v_max, double a_max, double magic_fabian_constant,
                                   double* values, uint8_t* fixed_mask, double* times,
                                   int threads);
/* createRandomVerticesPath (src/polynomial_timing_evaluation.cpp:34-91) +
 * estimateSegmentTimes(v_max, a_max, magic) as timeEval does (:93-112) */
int mtg_host_random_vertices_path_batch(int N, int D, int K, double average_distance,
                                        int max_derivative, uint32_t seed0, int64_t batch,
                                        double v_max, double a_max, double magic_fabian_constant,
                                        double* values, uint8_t* fixed_mask, double* times,
                                        int threads);

/* estimateSegmentTimes (src/vertex.cpp:162-178) on explicit positions [n_vertices][D]:
 * times[i] = 2 d / v_max (1 + magic v_max / a_max exp(-2 d / v_max)), d = |p_{i+1} - p_i| with
 * Eigen's norm reduction order.  times [n_vertices - 1]. */
int mtg_host_estimate_segment_times(int n_vertices, int D, const double* positions, double v_max, double a_max,
                                    double magic_fabian_constant, double* times);

/* Per-segment matrices of PolynomialOptimization<N> at segment time T (> 0), N x N row-major, any
 * pointer may be NULL:
 *   A      setupMappingMatrix (lin_impl:102-111)
 *   A_inv  A(T)^-1 (invertMappingMatrix, lin_impl:133-169), from the exact A(1)^-1 table:
 *          diag(T^-j) A(1)^-1 S(T), S = diag(T^(slot mod N/2))
 *   Q      computeQuadraticCostJacobian(derivative_to_optimize, T) (lin_impl:574-589)
 *   H      A^-T Q A^-1 (constructR's per-segment block, lin_impl:305-308), from the exact table:
 *          T^(1-2r) S Htilde S
 * They back getA / getAInverse / getR of the C++ drop-in. */
int mtg_host_segment_matrices(int N, int derivative_to_optimize, double T, double* A, double* A_inv, double* Q,
                              double* H);

/* Host form of mtg_coefficients_from_vertices_batch (setFreeConstraints +
 * updateSegmentsFromCompactConstraints, lin_impl:253-273) for the C++ drop-in's single problems:
 * vertex_values [B][V][h][D] (all derivatives), times [B][K] -> coeffs [B][K][D][N]. */
int mtg_host_coefficients_from_vertices_batch(int N, int D, int K, int64_t batch, const double* vertex_values,
                                              const double* times, double* coeffs, int threads);

#ifdef __cplusplus
}
#endif
#endif /* MTG_H_ */
