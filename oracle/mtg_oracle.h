/*
 * mtg_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * Plain-C restatement of the reference's CPU linear minimum-derivative solver
 * (magrimm/mav_trajectory_generation_cmake, "lin_impl" =
 * mav_trajectory_generation/include/mav_trajectory_generation/impl/
 * polynomial_optimization_linear_impl.h) and of the helpers on its path.
 * Every function cites the reference file:line it follows.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.  The
 * product path (libmav_trajectory_generation.so) never links or calls it.
 *
 * Parity pinning (see DESIGN.md "Oracle"): the reference needs Eigen3, glog
 * and nlopt, none present, so it cannot be compiled here.  This restatement is
 * pinned by the reference's own known-answer test (2_vertices_setup,
 * test/test_polynomial_optimization.cpp:700-744), its A-inversion test
 * (:194-204), its invariants (checkPath :73-131, ConstraintPacking :777-836,
 * checkCost :133-152), the C++ standard's mt19937 known answer, and 60-digit
 * mpmath truth fixtures (tests/golden/).
 *
 * Deliberate difference: Eigen::SparseQR<COLAMD> (lin_impl:355-364) is
 * replaced by a dense Householder QR of the same R_pp; both are backward
 * stable, rounding differs in the last digits.
 */
#ifndef MTG_ORACLE_H_
#define MTG_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_KMAXN 12
#define ORACLE_OK 0
#define ORACLE_ERR_ARG (-1)
#define ORACLE_ERR_BAD_DERIVATIVE (-3)
#define ORACLE_ERR_BAD_TIME (-4)
#define ORACLE_WARN_DROPPED 1

/* ---- libstdc++ <random> restatement (std::mt19937 + uniform_real_distribution) */
typedef struct {
  uint32_t mt[624];
  int idx;
} oracle_mt19937;
void oracle_mt_seed(oracle_mt19937* g, uint32_t seed);
uint32_t oracle_mt_next(oracle_mt19937* g);
double oracle_uniform(oracle_mt19937* g, double a, double b);

/* ---- polynomial.h / polynomial.cpp */
double oracle_base_coefficient(int n, int i);
void oracle_base_coeffs_with_time(int N, int derivative, double t, double* out);
double oracle_poly_evaluate(int N, const double* c, double t, int derivative);

/* ---- vertex.cpp / polynomial_timing_evaluation.cpp generators.
 * Output: values [V][nd][D] (derivative-major per vertex, zero where unset),
 * mask [V] (bit k => derivative k constrained).  nd must be > max_derivative. */
int oracle_create_random_vertices(int max_derivative, int K, int D, const double* pos_min,
                                  const double* pos_max, uint32_t seed, int nd, double* values,
                                  uint32_t* mask);
int oracle_create_random_vertices_path(int D, int K, double average_distance, int max_derivative,
                                       uint32_t seed, int nd, double* values, uint32_t* mask);
void oracle_estimate_segment_times(int K, int D, int nd, const double* values, double v_max,
                                   double a_max, double magic_fabian_constant, double* times);

/* ---- the linear solver.  Inputs: values [V][nd][D], mask [V], times [K]. */
typedef struct {
  int N, D, K, r, nd;
  const double* values;
  const uint32_t* mask;
  const double* times;
} oracle_problem;

/* Optional outputs (any pointer may be NULL):
 *   coeffs   [K][D][N]        increasing powers (polynomial_optimization_linear.h:42-44)
 *   fixed    [D][n_fixed]     getFixedConstraints order, free [D][n_free] getFreeConstraints
 *   col_of_row [n_all]        M as a row->column map (each row of M has one 1)
 *   ainv     [K][N][N], amap [K][N][N], qmat [K][N][N]
 *   cost     computeCost() (lin_impl:114-130)
 * Returns ORACLE_OK (| ORACLE_WARN_DROPPED when constraints > N/2-1 were dropped)
 * or a negative error.  counts[0..2] = n_all, n_fixed, n_free. */
typedef struct {
  double* coeffs;
  double* fixed;
  double* free_;
  int* col_of_row;
  double* ainv;
  double* amap;
  double* qmat;
  double* cost;
  int counts[3];
} oracle_outputs;

int oracle_solve_linear(const oracle_problem* p, oracle_outputs* out);

/* Static helpers of PolynomialOptimization<N> (lin_impl:102-111, :133-169, :574-589). */
void oracle_setup_mapping_matrix(int N, double T, double* A);
void oracle_invert_mapping_matrix(int N, const double* A, double* Ainv);
void oracle_quadratic_cost_jacobian(int N, int derivative, double T, double* Q);
/* getCostAndGradientDerivative (polynomial_optimization_nonlinear_impl.h:1452-1520) at candidate
 * times: J[b][c] = sum_dims d^T R(T_c) d with the reference's per-segment H = A^-T Q A^-1
 * (updateSegmentTimes lin_impl:276-295), T_c[i] = times[b][i] * scales[c][i].
 * xfull [B][V][nd][D] holds every derivative (fixed and solved free) of every vertex. */
int oracle_cost_at_times_batch(int N, int D, int K, int r, int nd, int64_t B, const double* xfull,
                               const double* times, int C, const double* scales, double* J,
                               int threads);
/* getCostAndGradientTime's J_d term (polynomial_optimization_nonlinear_impl.h:2172-2229) at the
 * same candidates: G[b][c][n] = central difference of J_d in T_n with increment_time (the
 * reference's 0.1 floor included), or the exact derivative (Richardson limit) for 0. */
int oracle_cost_time_jacobian_batch(int N, int D, int K, int r, int nd, int64_t B, const double* xfull,
                                    const double* times, int C, const double* scales, double increment_time,
                                    double* J, double* G, int threads);

/* Batched convenience for the CPU baseline: B problems with identical shape,
 * values [B][V][nd][D] etc.  Runs on `threads` OpenMP threads (<=0: all). */
int oracle_solve_linear_batch(int N, int D, int K, int r, int nd, int64_t B, const double* values,
                              const uint32_t* mask, const double* times, double* coeffs,
                              double* cost, int threads);

/* ---- trajectory.cpp:68-128  Trajectory::evaluateRange (incl. its quirk that
 * sampling times restart at the start segment's beginning).  coeffs [K][D][N].
 * Writes at most max_samples rows of out [.][D] and times; returns the number
 * of samples the reference would produce (may exceed max_samples). */
int64_t oracle_evaluate_range(int N, int D, int K, const double* coeffs, const double* times,
                              double t_start, double t_end, double dt, int derivative,
                              int64_t max_samples, double* out, double* sample_times);

#ifdef __cplusplus
}
#endif
#endif /* MTG_ORACLE_H_ */
