// polynomial_optimization_linear.h -- PolynomialOptimization<N>, the drop-in for the reference's
// linear minimum-derivative optimizer (reference polynomial_optimization_linear.h:46-269 and
// impl/polynomial_optimization_linear_impl.h, "lin_impl" below).
//
// Same class, method names, argument meaning and CHECK behaviour (runtime.h).  What differs is how
// the problem is solved: R = M^T A^-T Q A^-1 M is never formed and no sparse QR runs.  The library
// (include/mtg.h) solves the block-tridiagonal system of the (vertex, derivative) unknowns with
// fixed derivatives pinned, by block LDL^T Thomas elimination on exact-rational per-segment tables
// -- in hand-written HIP for batches (BatchPolynomialOptimization<N>, batch_polynomial_optimization.h)
// and in its host solver for the single problem this class holds (ExecutionPolicy, runtime.h).
// The matrices the reference exposes (getA/getAInverse/getM/getR/getMpinv) are built on request.
//
// Requires C++17 and N even in [2, 12] (the reference's own limit is kMaxN = 12, polynomial.h:46).
// setupFromPositons (declared at polynomial_optimization_linear.h:79 but never defined by the
// reference) is not provided.
#ifndef MAV_TRAJECTORY_GENERATION_POLYNOMIAL_OPTIMIZATION_LINEAR_H_
#define MAV_TRAJECTORY_GENERATION_POLYNOMIAL_OPTIMIZATION_LINEAR_H_

#include <algorithm>
#include <cmath>
#include <limits>
#include <ostream>
#include <string>
#include <utility>
#include <vector>

#include "mav_trajectory_generation/extremum.h"
#include "mav_trajectory_generation/linalg.h"
#include "mav_trajectory_generation/motion_defines.h"
#include "mav_trajectory_generation/polynomial.h"
#include "mav_trajectory_generation/runtime.h"
#include "mav_trajectory_generation/segment.h"
#include "mav_trajectory_generation/trajectory.h"
#include "mav_trajectory_generation/vertex.h"

namespace mav_trajectory_generation {

namespace detail {
// Real roots of sum_j c_j t^j in [t0, t1]: sign changes on 256 uniform samples, each bracket
// refined by safeguarded Newton-bisection.  (The reference uses Jenkins-Traub, src/rpoly.cpp, which
// is outside the ported path; the GPU extrema kernel, mtg_extrema.hip, isolates roots the same
// way.)  A root pair closer than (t1 - t0)/256 without a sign change between samples is not found.
inline void real_roots_in(const VectorXd& c, double t0, double t1, std::vector<double>* roots) {
  const int n = (int)c.size();
  auto f = [&](double t) {
    double r = 0.0;
    for (int j = n - 1; j >= 0; --j) r = r * t + c[j];
    return r;
  };
  auto df = [&](double t) {
    double r = 0.0;
    for (int j = n - 1; j >= 1; --j) r = r * t + j * c[j];
    return r;
  };
  bool any = false;
  for (int j = 1; j < n; ++j) any = any || c[j] != 0.0;
  if (!any || !(t1 >= t0)) return;
  constexpr int kSamples = 256;
  double ta = t0, fa = f(t0);
  for (int s = 1; s <= kSamples; ++s) {
    const double tb = s == kSamples ? t1 : t0 + (t1 - t0) * s / kSamples;
    const double fb = f(tb);
    if (fa == 0.0) {
      roots->push_back(ta);
    } else if ((fa < 0.0) != (fb < 0.0) && fb != 0.0) {
      double lo = ta, hi = tb, flo = fa, t = 0.5 * (ta + tb);
      for (int it = 0; it < 100; ++it) {
        const double ft = f(t);
        if (ft == 0.0) break;
        if ((ft < 0.0) == (flo < 0.0)) lo = t, flo = ft;
        else hi = t;
        const double d = df(t);
        double tn = d != 0.0 ? t - ft / d : 0.5 * (lo + hi);
        if (!(tn > lo && tn < hi)) tn = 0.5 * (lo + hi);
        if (std::fabs(tn - t) <= 4.0 * std::numeric_limits<double>::epsilon() * std::fabs(t) || hi - lo == 0.0) {
          t = tn;
          break;
        }
        t = tn;
      }
      roots->push_back(t);
    }
    ta = tb;
    fa = fb;
  }
  if (fa == 0.0) roots->push_back(t1);
}
}  // namespace detail

template <int _N = 10>
class PolynomialOptimization {
  static_assert(_N % 2 == 0, "The number of coefficients has to be even.");
  static_assert(_N >= 2 && _N <= 12, "N must be in [2, 12] (Polynomial::kMaxN)");

 public:
  enum { N = _N };
  static constexpr int kHighestDerivativeToOptimize = N / 2 - 1;
  typedef FixedMatrix<N, N> SquareMatrix;
  // polynomial_optimization_linear.h:53-54: Eigen's aligned allocator (std::allocator without Eigen)
  typedef std::vector<SquareMatrix, AlignedAllocator<SquareMatrix>> SquareMatrixVector;

  // lin_impl:33-44
  explicit PolynomialOptimization(size_t dimension)
      : dimension_(dimension),
        derivative_to_optimize_(derivative_order::kINVALID),
        n_vertices_(0),
        n_segments_(0),
        n_all_constraints_(0),
        n_fixed_constraints_(0),
        n_free_constraints_(0) {
    fixed_constraints_compact_.resize(dimension_);
    free_constraints_compact_.resize(dimension_);
  }

  // lin_impl:47-99: copy the problem, drop constraints of order > N/2-1 with a warning, set up the
  // segment times and the (vertex, derivative) ordering of fixed and free constraints.
  bool setupFromVertices(const Vertex::Vector& vertices, const std::vector<double>& segment_times,
                         int derivative_to_optimize = kHighestDerivativeToOptimize) {
    if (derivative_to_optimize < 0 || derivative_to_optimize > kHighestDerivativeToOptimize)
      fail(MTG_ERR_BAD_DERIVATIVE, "You tried to optimize the " + std::to_string(derivative_to_optimize) +
                                       "th derivative of position on a " + std::to_string(N) +
                                       "th order polynomial. This is not possible.");
    if (vertices.size() != segment_times.size() + 1)
      fail(MTG_ERR_SIZE_MISMATCH, "Size of times must be one less than positions.");
    derivative_to_optimize_ = derivative_to_optimize;
    vertices_ = vertices;
    n_vertices_ = vertices_.size();
    n_segments_ = n_vertices_ - 1;
    segments_.assign(n_segments_, Segment(N, (int)dimension_));
    for (size_t v = 0; v < n_vertices_; ++v) {
      Vertex& vertex = vertices_[v];
      if (vertex.D() != (int)dimension_) fail(MTG_ERR_SIZE_MISMATCH, "vertex dimension mismatch");
      bool valid = true;  // (lin_impl:74-95; the vertex is rebuilt only when it must drop something)
      for (auto it = vertex.cBegin(); it != vertex.cEnd(); ++it) valid = valid && it->first <= kHighestDerivativeToOptimize;
      if (!valid) {
        Vertex tmp(dimension_);
        for (auto it = vertex.cBegin(); it != vertex.cEnd(); ++it) {
          if (it->first > kHighestDerivativeToOptimize) {
            warn("Invalid constraint on vertex " + std::to_string(v) + ": maximum possible derivative is " +
                 std::to_string(kHighestDerivativeToOptimize) + ", but was set to " + std::to_string(it->first) +
                 ". Ignoring constraint");
          } else {
            tmp.addConstraint(it->first, it->second);
          }
        }
        vertex = tmp;
      }
    }
    updateSegmentTimes(segment_times);
    setupConstraintReorderingMatrix();
    return true;
  }

  // A^-1 by the Schur complement of A's block structure [A_diag 0; C D] (lin_impl:133-169), for any
  // mapping matrix with that structure (the h x h D block inverted with partial pivoting).
  static void invertMappingMatrix(const SquareMatrix& mapping_matrix, SquareMatrix* inverse_mapping_matrix) {
    check_notnull(inverse_mapping_matrix, "inverse_mapping_matrix");
    constexpr int h = N / 2;
    double Ad[h], Dm[h][h], Di[h][h], C[h][h];
    for (int i = 0; i < h; ++i) {
      Ad[i] = 1.0 / mapping_matrix(i, i);
      for (int j = 0; j < h; ++j) {
        C[i][j] = mapping_matrix(h + i, j);
        Dm[i][j] = mapping_matrix(h + i, h + j);
        Di[i][j] = i == j ? 1.0 : 0.0;
      }
    }
    for (int c = 0; c < h; ++c) {  // Gauss-Jordan with partial pivoting on D
      int p = c;
      for (int r = c + 1; r < h; ++r)
        if (std::fabs(Dm[r][c]) > std::fabs(Dm[p][c])) p = r;
      for (int j = 0; j < h; ++j) std::swap(Dm[c][j], Dm[p][j]), std::swap(Di[c][j], Di[p][j]);
      const double inv = 1.0 / Dm[c][c];
      for (int j = 0; j < h; ++j) Dm[c][j] *= inv, Di[c][j] *= inv;
      for (int r = 0; r < h; ++r) {
        if (r == c || Dm[r][c] == 0.0) continue;
        const double f = Dm[r][c];
        for (int j = 0; j < h; ++j) Dm[r][j] -= f * Dm[c][j], Di[r][j] -= f * Di[c][j];
      }
    }
    SquareMatrix& out = *inverse_mapping_matrix;
    for (int i = 0; i < h; ++i)
      for (int j = 0; j < h; ++j) {
        out(i, j) = i == j ? Ad[i] : 0.0;
        out(i, h + j) = 0.0;
        out(h + i, h + j) = Di[i][j];
        double t = 0.0;  // -(D^-1 C A_diag^-1)
        for (int k = 0; k < h; ++k) t += Di[i][k] * C[k][j];
        out(h + i, j) = -t * Ad[j];
      }
  }

  // A = [rows of derivative k at t = 0; at t = segment_time] (lin_impl:102-111)
  static void setupMappingMatrix(double segment_time, SquareMatrix* A) {
    check_notnull(A, "A");
    for (int i = 0; i < N / 2; ++i) {
      const VectorXd r0 = Polynomial::baseCoeffsWithTime(N, i, 0.0);
      const VectorXd r1 = Polynomial::baseCoeffsWithTime(N, i, segment_time);
      for (int j = 0; j < N; ++j) (*A)(i, j) = r0[j], (*A)(i + N / 2, j) = r1[j];
    }
  }

  // 0.5 sum_i sum_d c^T Q_i c over the current segments and segment times (lin_impl:114-130)
  double computeCost() const {
    double cost = 0.0;
    for (size_t i = 0; i < n_segments_; ++i) {
      SquareMatrix Q;
      computeQuadraticCostJacobian(derivative_to_optimize_, segment_times_[i], &Q);
      for (size_t d = 0; d < dimension_; ++d) {
        const VectorXd c = segments_[i][d].getCoefficients(derivative_order::POSITION);
        double part = 0.0;
        for (int a = 0; a < N; ++a) {
          double row = 0.0;
          for (int b = 0; b < N; ++b) row += Q(a, b) * c[b];
          part += c[a] * row;
        }
        cost += part;
      }
    }
    return 0.5 * cost;
  }

  // lin_impl:276-295
  void updateSegmentTimes(const std::vector<double>& segment_times) {
    if (segment_times.size() != n_segments_)
      fail(MTG_ERR_SIZE_MISMATCH, "Number of segment times (" + std::to_string(segment_times.size()) +
                                      ") does not match number of segments (" + std::to_string(n_segments_) + ")");
    for (double t : segment_times)
      if (!(t > 0)) fail(MTG_ERR_INVALID_ARGUMENT, "Segment times need to be greater than zero");
    segment_times_ = segment_times;
  }

  // lin_impl:329-369.  n_free == 0 outputs the fully constrained polynomials with a warning (:333-339).
  bool solveLinear() {
    if (derivative_to_optimize_ < 0 || derivative_to_optimize_ > kHighestDerivativeToOptimize)
      fail(MTG_ERR_BAD_DERIVATIVE, "solveLinear before setupFromVertices");
    if (n_free_constraints_ == 0)
      warn("No free constraints set in the vertices. Polynomial can not be optimized. Outputting fully "
           "constrained polynomial.");
    const int K = (int)n_segments_, D = (int)dimension_, V = K + 1, h = N / 2;
    std::vector<double> coeffs((size_t)K * D * N), free((size_t)D * V * h);
    int32_t nfree = 0, status = 0;
    double cost = 0.0;
    if (singleOnDevice()) {
      mtg_ctx* ctx = defaultContext();
      check(mtg_solve_linear_batch(ctx, N, D, K, derivative_to_optimize_, 1, values_.data(), mask_.data(),
                                   segment_times_.data(), coeffs.data(), free.data(), &nfree, &cost, &status, 0),
            ctx, "mtg_solve_linear_batch");
    } else {
      check(mtg_host_solve_linear_batch(N, D, K, derivative_to_optimize_, 1, values_.data(), mask_.data(),
                                        segment_times_.data(), coeffs.data(), free.data(), &nfree, &cost,
                                        &status, 1),
            nullptr, "mtg_host_solve_linear_batch");
    }
    if (status & MTG_TRAJ_BAD_TIME) fail(MTG_ERR_INVALID_ARGUMENT, "Segment times need to be greater than zero");
    if (status & MTG_TRAJ_NOT_SPD) warn("R_pp is not positive definite: the solution is not reliable");
    for (int d = 0; d < D; ++d) {
      VectorXd f(n_free_constraints_);
      for (size_t i = 0; i < n_free_constraints_; ++i) f[i] = free[(size_t)d * V * h + i];
      free_constraints_compact_[d] = f;
    }
    setSegmentsFromCoefficients(coeffs);
    return true;
  }

  void getTrajectory(Trajectory* trajectory) const { check_notnull(trajectory, "trajectory")->setSegments(segments_); }

  // Roots in [t_start, t_stop] of sum_d conv(p_d^(Derivative), p_d^(Derivative+1)) (one dimension:
  // of p^(Derivative+1)), the magnitude's stationary points (lin_impl:377-433).
  template <int Derivative>
  static bool computeSegmentMaximumMagnitudeCandidates(const Segment& segment, double t_start, double t_stop,
                                                       std::vector<double>* candidates) {
    check_notnull(candidates, "candidates");
    static_assert(N - Derivative - 1 > 0, "N-Derivative-1 has to be greater 0");
    constexpr int n_d = N - Derivative, n_dd = N - Derivative - 1;
    VectorXd f;
    if (segment.D() > 1) {
      f = VectorXd::Zero(n_d + n_dd - 1);
      for (const Polynomial& p : segment.getPolynomialsRef())
        f += Polynomial::convolve(p.getCoefficients(Derivative).head(n_d), p.getCoefficients(Derivative + 1).head(n_dd));
    } else {
      f = segment[0].getCoefficients(Derivative + 1).head(n_dd);
    }
    detail::real_roots_in(f, t_start, t_stop, candidates);
    return true;
  }

  // Candidates by sampling (lin_impl:435-466; debugging / testing).
  template <int Derivative>
  static void computeSegmentMaximumMagnitudeCandidatesBySampling(const Segment& segment, double t_start,
                                                                 double t_stop, double dt,
                                                                 std::vector<double>* candidates) {
    check_notnull(candidates, "candidates");
    auto sgn = [](double x) { return (x > 0.0) - (x < 0.0); };
    const VectorXd value_start = segment.evaluate(t_start - dt, Derivative);
    VectorXd value_old = segment.evaluate(t_start, Derivative);
    double direction = value_old.squaredNorm() - value_start.squaredNorm();
    for (double t = t_start + dt; t < t_stop + 2 * dt; t += dt) {
      const VectorXd value_new = segment.evaluate(t, Derivative);
      const double direction_new = value_new.squaredNorm() - value_old.squaredNorm();
      if (sgn(direction) != sgn(direction_new)) candidates->push_back(t - dt);
      value_old = value_new;
      direction = direction_new;
    }
  }

  // Largest magnitude of the Derivative over the trajectory: segment starts, stationary points and
  // the final time (lin_impl:468-503).
  template <int Derivative>
  Extremum computeMaximumOfMagnitude(std::vector<Extremum>* candidates) const {
    if (candidates != nullptr) candidates->clear();
    int segment_idx = 0;
    Extremum extremum;
    for (const Segment& s : segments_) {
      std::vector<double> extrema_times;
      extrema_times.reserve(N - 1);
      extrema_times.push_back(0.0);
      computeSegmentMaximumMagnitudeCandidates<Derivative>(s, 0.0, s.getTime(), &extrema_times);
      for (double t : extrema_times) {
        const Extremum candidate(t, s.evaluate(t, Derivative).norm(), segment_idx);
        if (extremum < candidate) extremum = candidate;
        if (candidates != nullptr) candidates->emplace_back(candidate);
      }
      ++segment_idx;
    }
    const Extremum candidate(segments_.back().getTime(),
                             segments_.back().evaluate(segments_.back().getTime(), Derivative).norm(),
                             (int)n_segments_ - 1);
    if (extremum < candidate) extremum = candidate;
    if (candidates != nullptr) candidates->emplace_back(candidate);
    return extremum;
  }

  void getSegments(Segment::Vector* segments) const { *check_notnull(segments, "segments") = segments_; }
  void getSegmentTimes(std::vector<double>* segment_times) const {
    *check_notnull(segment_times, "segment_times") = segment_times_;
  }
  void getFreeConstraints(std::vector<VectorXd>* free_constraints) const {
    *check_notnull(free_constraints, "free_constraints") = free_constraints_compact_;
  }
  void getFixedConstraints(std::vector<VectorXd>* fixed_constraints) const {
    *check_notnull(fixed_constraints, "fixed_constraints") = fixed_constraints_compact_;
  }

  // New free derivatives (per dimension, the getFreeConstraints order); the segments follow
  // (lin_impl:505-514 + updateSegmentsFromCompactConstraints :253-273).
  void setFreeConstraints(const std::vector<VectorXd>& free_constraints) {
    if (free_constraints.size() != dimension_) fail(MTG_ERR_SIZE_MISMATCH, "setFreeConstraints: dimension mismatch");
    for (const VectorXd& v : free_constraints)
      if ((size_t)v.size() != n_free_constraints_) fail(MTG_ERR_SIZE_MISMATCH, "setFreeConstraints: size mismatch");
    free_constraints_compact_ = free_constraints;
    updateSegmentsFromCompactConstraints();
  }

  // Q_ij = 2 B(r, i) B(r, j) t^(i+j-2r+1) / (i+j-2r+1), i, j >= r (lin_impl:574-589)
  static void computeQuadraticCostJacobian(int derivative, double t, SquareMatrix* cost_jacobian) {
    check_notnull(cost_jacobian, "cost_jacobian");
    if (derivative >= N) fail(MTG_ERR_BAD_DERIVATIVE, "derivative must be < N");
    SquareMatrix& Q = *cost_jacobian;
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) Q(i, j) = 0.0;
    for (int col = 0; col < N - derivative; col++)
      for (int row = 0; row < N - derivative; row++) {
        const double exponent = (N - 1 - derivative) * 2 + 1 - row - col;
        Q(N - 1 - row, N - 1 - col) = Polynomial::base_coefficients_(derivative, N - 1 - row) *
                                      Polynomial::base_coefficients_(derivative, N - 1 - col) *
                                      std::pow(t, exponent) * 2.0 / exponent;
      }
  }

  size_t getDimension() const { return dimension_; }
  size_t getNumberSegments() const { return n_segments_; }
  size_t getNumberAllConstraints() const { return n_all_constraints_; }
  size_t getNumberFixedConstraints() const { return n_fixed_constraints_; }
  size_t getNumberFreeConstraints() const { return n_free_constraints_; }
  int getDerivativeToOptimize() const { return derivative_to_optimize_; }
  void getVertices(Vertex::Vector* vertices) const { *check_notnull(vertices, "vertices") = vertices_; }

  // Block diagonal of the per-segment A^-1 (lin_impl:517-527), from the exact A(1)^-1 table.
  void getAInverse(MatrixXd* A_inv) const {
    check_notnull(A_inv, "A_inv");
    const Index n = (Index)(N * n_segments_);
    A_inv->resize(n, n);
    A_inv->setZero();
    std::vector<double> Ai((size_t)N * N);
    for (size_t i = 0; i < n_segments_; ++i) {
      check(mtg_host_segment_matrices(N, 0, segment_times_[i], nullptr, Ai.data(), nullptr, nullptr), nullptr,
            "mtg_host_segment_matrices");
      for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b) (*A_inv)((Index)(i * N + a), (Index)(i * N + b)) = Ai[(size_t)a * N + b];
    }
  }
  // The 0/1 reordering matrix (C in [1]): row i*N + s is segment i's slot s (vertex i + (s >= N/2),
  // derivative s mod N/2), column its rank among fixed-then-free sorted constraints (lin_impl:172-250).
  void getM(MatrixXd* M) const {
    check_notnull(M, "M")->resize((Index)n_all_constraints_, (Index)(n_fixed_constraints_ + n_free_constraints_));
    M->setZero();
    for (size_t row = 0; row < col_of_row_.size(); ++row) (*M)((Index)row, (Index)col_of_row_[row]) = 1.0;
  }
  // R = M^T blkdiag(A^-T Q A^-1) M (constructR, lin_impl:298-326), per-segment blocks from the exact
  // Htilde table.
  void getR(MatrixXd* R) const {
    check_notnull(R, "R");
    const size_t n = n_fixed_constraints_ + n_free_constraints_;
    R->resize((Index)n, (Index)n);
    R->setZero();
    std::vector<double> H((size_t)N * N);
    for (size_t i = 0; i < n_segments_; ++i) {
      check(mtg_host_segment_matrices(N, derivative_to_optimize_, segment_times_[i], nullptr, nullptr, nullptr,
                                      H.data()),
            nullptr, "mtg_host_segment_matrices");
      for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b)
          (*R)((Index)col_of_row_[i * N + a], (Index)col_of_row_[i * N + b]) += H[(size_t)a * N + b];
    }
  }
  // Block diagonal of the per-segment mapping matrices A (lin_impl:545-560).
  void getA(MatrixXd* A) const {
    check_notnull(A, "A");
    const Index n = (Index)(N * n_segments_);
    A->resize(n, n);
    A->setZero();
    for (size_t i = 0; i < n_segments_; ++i) {
      if (!(segment_times_[i] > 0)) fail(MTG_ERR_INVALID_ARGUMENT, "Segment times need to be greater than zero");
      SquareMatrix As;
      setupMappingMatrix(segment_times_[i], &As);
      for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b) (*A)((Index)(i * N + a), (Index)(i * N + b)) = As(a, b);
    }
  }
  // M^T with each row divided by its sum: the pseudo-inverse of the 0/1 M (lin_impl:562-571).
  void getMpinv(MatrixXd* M_pinv) const {
    check_notnull(M_pinv, "M_pinv");
    MatrixXd M;
    getM(&M);
    *M_pinv = M.transpose();
    for (Index r = 0; r < M_pinv->rows(); ++r) {
      double s = 0.0;
      for (Index c = 0; c < M_pinv->cols(); ++c) s += (*M_pinv)(r, c);
      for (Index c = 0; c < M_pinv->cols(); ++c) (*M_pinv)(r, c) /= s;
    }
  }

  void printReorderingMatrix(std::ostream& stream) const {
    MatrixXd M;
    getM(&M);
    stream << "Mapping matrix:\n" << M << std::endl;
  }

 private:
  // Constraint bookkeeping of setupConstraintReorderingMatrix (lin_impl:172-250) in the ABI layout:
  // values_ [V][h][D] / mask_ [V] (bit k: derivative k fixed), the row -> column map of M, and the
  // compact fixed values per dimension.  Fixed columns come first, each set sorted by (vertex,
  // derivative) (Constraint::operator<, polynomial_optimization_linear.h:273-280).
  void setupConstraintReorderingMatrix() {
    const int h = N / 2, D = (int)dimension_, V = (int)n_vertices_;
    values_.assign((size_t)V * h * D, 0.0);
    mask_.assign(V, 0);
    std::vector<int> fixed_rank((size_t)V * h, -1), free_rank((size_t)V * h, -1);
    int nf = 0, np = 0;
    for (int v = 0; v < V; ++v) {
      // the vertex's constraints in derivative order (a std::map), read in place
      auto it = vertices_[v].cBegin();
      const auto end = vertices_[v].cEnd();
      for (int k = 0; k < h; ++k) {
        while (it != end && it->first < k) ++it;
        if (it != end && it->first == k) {
          mask_[v] |= (uint8_t)(1u << k);
          for (int d = 0; d < D; ++d) values_[((size_t)v * h + k) * D + d] = it->second[d];
          fixed_rank[(size_t)v * h + k] = nf++;
        } else {
          free_rank[(size_t)v * h + k] = np++;
        }
      }
    }
    n_fixed_constraints_ = nf;
    n_free_constraints_ = np;
    n_all_constraints_ = (size_t)N * n_segments_;  // ends once, interior vertices twice
    col_of_row_.assign(n_all_constraints_, 0);
    for (size_t i = 0; i < n_segments_; ++i)
      for (int s = 0; s < N; ++s) {
        const size_t vk = (i + (s >= h ? 1 : 0)) * h + (s % h);
        col_of_row_[i * N + s] = fixed_rank[vk] >= 0 ? fixed_rank[vk] : nf + free_rank[vk];
      }
    for (int d = 0; d < D; ++d) {
      VectorXd f(nf);
      int idx = 0;
      for (int v = 0; v < V; ++v)
        for (int k = 0; k < h; ++k)
          if ((mask_[v] >> k) & 1u) f[idx++] = values_[((size_t)v * h + k) * D + d];
      fixed_constraints_compact_[d] = f;
    }
  }

  // c_i = A_i^-1 (M [d_f; d_p])_i for every segment and dimension (lin_impl:253-273)
  void updateSegmentsFromCompactConstraints() {
    const int h = N / 2, D = (int)dimension_, V = (int)n_vertices_, K = (int)n_segments_;
    std::vector<double> x((size_t)V * h * D, 0.0), coeffs((size_t)K * D * N);
    for (int d = 0; d < D; ++d) {
      int idx = 0;
      for (int v = 0; v < V; ++v)
        for (int k = 0; k < h; ++k) {
          const size_t o = ((size_t)v * h + k) * D + d;
          x[o] = ((mask_[v] >> k) & 1u) ? values_[o] : free_constraints_compact_[d][idx++];
        }
    }
    if (singleOnDevice()) {
      mtg_ctx* ctx = defaultContext();
      check(mtg_coefficients_from_vertices_batch(ctx, N, D, K, 1, x.data(), segment_times_.data(), coeffs.data(), 0),
            ctx, "mtg_coefficients_from_vertices_batch");
    } else {
      check(mtg_host_coefficients_from_vertices_batch(N, D, K, 1, x.data(), segment_times_.data(), coeffs.data(), 1),
            nullptr, "mtg_host_coefficients_from_vertices_batch");
    }
    setSegmentsFromCoefficients(coeffs);
  }

  // (the segments' polynomials, order N since setupFromVertices, take the coefficients into their own
  // storage: one buffer per call instead of a vector and a polynomial per segment and dimension)
  void setSegmentsFromCoefficients(const std::vector<double>& coeffs) {
    const int D = (int)dimension_;
    VectorXd c(N);
    for (size_t i = 0; i < n_segments_; ++i) {
      Segment& s = segments_[i];
      s.setTime(segment_times_[i]);
      for (int d = 0; d < D; ++d) {
        for (int j = 0; j < N; ++j) c[j] = coeffs[(i * D + d) * N + j];
        s[d].setCoefficients(c);
      }
    }
  }

  Vertex::Vector vertices_;
  Segment::Vector segments_;
  std::vector<VectorXd> fixed_constraints_compact_;
  std::vector<VectorXd> free_constraints_compact_;
  std::vector<double> segment_times_;
  size_t dimension_;
  int derivative_to_optimize_;
  size_t n_vertices_;
  size_t n_segments_;
  size_t n_all_constraints_;
  size_t n_fixed_constraints_;
  size_t n_free_constraints_;
  std::vector<double> values_;     // [V][h][D] fixed values (ABI layout)
  std::vector<uint8_t> mask_;      // [V]
  std::vector<size_t> col_of_row_;  // M as a row -> column map
};

// PolynomialOptimizationNonLinear::computeInitialSolutionWithoutPositionConstraints
// (polynomial_optimization_nonlinear_impl.h:116-187) on a linear problem: solve, remove the
// position constraint of every interior vertex, set the problem up again with the same times and
// start its free derivatives from the solved trajectory (M^+ A p: the derivatives at the segment
// ends, averaged where two segments meet).  The polynomials are unchanged up to rounding; the
// free vector now holds the interior positions too.
template <int N>
bool computeInitialSolutionWithoutPositionConstraints(PolynomialOptimization<N>* opt) {
  check_notnull(opt, "opt");
  opt->solveLinear();
  Segment::Vector segments;
  opt->getSegments(&segments);
  std::vector<double> times;
  opt->getSegmentTimes(&times);
  Vertex::Vector vertices;
  opt->getVertices(&vertices);
  const int K = (int)times.size(), D = (int)opt->getDimension(), h = N / 2, V = K + 1;
  std::vector<double> x((size_t)V * h * D, 0.0);
  if (singleOnDevice()) {
    std::vector<double> coeffs((size_t)K * D * N);
    for (int i = 0; i < K; ++i)
      for (int d = 0; d < D; ++d) {
        const VectorXd c = segments[i][d].getCoefficients();
        for (int j = 0; j < N; ++j) coeffs[((size_t)i * D + d) * N + j] = c[j];
      }
    mtg_ctx* ctx = defaultContext();
    check(mtg_vertex_derivatives_batch(ctx, N, D, K, 1, coeffs.data(), times.data(), x.data(), 0), ctx,
          "mtg_vertex_derivatives_batch");
  } else {
    for (int v = 0; v < V; ++v) {
      const int n_ends = (v == 0 || v == K) ? 1 : 2;
      for (int k = 0; k < h; ++k)
        for (int d = 0; d < D; ++d) {
          double acc = 0.0;
          if (v > 0) acc += segments[v - 1][d].evaluate(segments[v - 1].getTime(), k);
          if (v < K) acc += segments[v][d].evaluate(0.0, k);
          x[((size_t)v * h + k) * D + d] = acc / n_ends;
        }
    }
  }
  for (int v = 1; v < V - 1; ++v) vertices[v].removeConstraint(derivative_order::POSITION);
  opt->setupFromVertices(vertices, times, opt->getDerivativeToOptimize());
  std::vector<VectorXd> free(D, VectorXd(opt->getNumberFreeConstraints()));
  for (int d = 0; d < D; ++d) {
    int idx = 0;
    for (int v = 0; v < V; ++v)
      for (int k = 0; k < h; ++k)
        if (!vertices[v].hasConstraint(k)) free[d][idx++] = x[((size_t)v * h + k) * D + d];
  }
  opt->setFreeConstraints(free);
  return true;
}

}  // namespace mav_trajectory_generation

#endif  // MAV_TRAJECTORY_GENERATION_POLYNOMIAL_OPTIMIZATION_LINEAR_H_
