// trajectory_generation.hpp -- C++17 drop-in surface of the reference's linear polynomial
// optimizer, implemented on the C ABI (mtg.h, libmtg.so).  Header-only; link with -lmtg.
//
// Mirrors (same names, argument meaning and error behaviour; Eigen vectors are std::vector<double>
// because this image has no Eigen -- INTEGRATION.md shows the Eigen adapter):
//   Vertex                          mav_trajectory_generation/include/.../vertex.h:42-107
//   Segment, Polynomial             segment.h:37-110, polynomial.h:42-233
//   Trajectory (evaluate, evaluateRange)   trajectory.h:32-140, src/trajectory.cpp:41-128
//   PolynomialOptimization<N>       polynomial_optimization_linear.h:46-269
// plus BatchPolynomialOptimization<N>, the batched entry point the GPU exists for.
//
// Error behaviour: the reference CHECK-fails (aborts) on a bad derivative_to_optimize
// (lin_impl:50-55), mismatched sizes (:66-67) and non-positive segment times (:287); so does this
// header, unless MTG_CPP_THROW is defined, in which case it throws mtg::Error.  Derivative orders
// above N/2-1 are dropped with a warning on stderr (LOG(WARNING), lin_impl:84-87).  The solve
// itself always runs on the GPU: without a HIP device every call fails (there is no CPU path).
#pragma once

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "mtg.h"

namespace mtg {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

[[noreturn]] inline void fail(int code, const std::string& what) {
#ifdef MTG_CPP_THROW
  throw Error(code, what);
#else
  std::fprintf(stderr, "mtg: check failed: %s (%s)\n", what.c_str(), mtg_status_string(code));
  std::abort();
#endif
}

inline void check(int rc, mtg_ctx* ctx, const char* where) {
  if (rc != MTG_OK) {
    std::string msg = where;
    const char* detail = ctx ? mtg_last_error(ctx) : nullptr;
    if (detail && *detail) msg += std::string(": ") + detail;
    fail(rc, msg);
  }
}

// One process-wide context on device 0 for the single-trajectory API (lazily created).
inline mtg_ctx* default_context() {
  static std::once_flag once;
  static mtg_ctx* ctx = nullptr;
  std::call_once(once, [] { check(mtg_create(0, &ctx), nullptr, "mtg_create(0)"); });
  return ctx;
}

namespace derivative_order {  // vertex.h / motion_defines.h
constexpr int POSITION = 0, VELOCITY = 1, ACCELERATION = 2, JERK = 3, SNAP = 4;
constexpr int ORIENTATION = 0, ANGULAR_VELOCITY = 1, ANGULAR_ACCELERATION = 2, INVALID = -1;
}  // namespace derivative_order

// ------------------------------------------------------------------------------------ Vertex
class Vertex {
 public:
  typedef std::vector<Vertex> Vector;
  typedef std::vector<double> ConstraintValue;
  typedef std::map<int, ConstraintValue> Constraints;

  explicit Vertex(size_t dimension) : D_(static_cast<int>(dimension)) {}
  int D() const { return D_; }
  void addConstraint(int derivative_order, double value) {
    constraints_[derivative_order] = ConstraintValue(D_, value);
  }
  void addConstraint(int derivative_order, const ConstraintValue& c) {
    if ((int)c.size() != D_) fail(MTG_ERR_SIZE_MISMATCH, "Vertex::addConstraint: dimension mismatch");
    constraints_[derivative_order] = c;
  }
  bool removeConstraint(int derivative_order) { return constraints_.erase(derivative_order) > 0; }
  void makeStartOrEnd(const ConstraintValue& c, int up_to_derivative) {  // src/vertex.cpp:106-112
    addConstraint(derivative_order::POSITION, c);
    for (int i = 1; i <= up_to_derivative; ++i) constraints_[i] = ConstraintValue(D_, 0.0);
  }
  void makeStartOrEnd(double value, int up_to_derivative) { makeStartOrEnd(ConstraintValue(D_, value), up_to_derivative); }
  bool hasConstraint(int derivative_order) const { return constraints_.count(derivative_order) > 0; }
  bool getConstraint(int derivative_order, ConstraintValue* c) const {
    auto it = constraints_.find(derivative_order);
    if (it == constraints_.end()) return false;
    if (c) *c = it->second;
    return true;
  }
  Constraints::const_iterator cBegin() const { return constraints_.begin(); }
  Constraints::const_iterator cEnd() const { return constraints_.end(); }
  size_t getNumberOfConstraints() const { return constraints_.size(); }

 private:
  int D_;
  Constraints constraints_;
};

// -------------------------------------------------------------------- Polynomial / Segment
class Polynomial {
 public:
  typedef std::vector<Polynomial> Vector;
  explicit Polynomial(int N) : c_(N, 0.0) {}
  explicit Polynomial(std::vector<double> coefficients) : c_(std::move(coefficients)) {}
  int N() const { return (int)c_.size(); }
  const std::vector<double>& getCoefficients() const { return c_; }
  // Horner on B(d, j) c_j, multiply-then-add (polynomial.h:138-151)
  double evaluate(double t, int derivative) const {
    const int n = N();
    if (derivative >= n) return 0.0;
    double r = base(derivative, n - 1) * c_[n - 1];
    for (int j = n - 2; j >= derivative; --j) {
      r *= t;
      r += base(derivative, j) * c_[j];
    }
    return r;
  }
  static double base(int d, int i) {  // i! / (i - d)!  (src/polynomial.cpp:140-155)
    if (i < d) return 0.0;
    double out = 1.0;
    for (int k = i - d + 1; k <= i; ++k) out *= (double)k;
    return out;
  }

 private:
  std::vector<double> c_;
};

class Segment {
 public:
  typedef std::vector<Segment> Vector;
  Segment(int N, int D) : N_(N), D_(D), polynomials_(D, Polynomial(N)) {}
  int D() const { return D_; }
  int N() const { return N_; }
  double getTime() const { return time_; }
  void setTime(double t) { time_ = t; }
  Polynomial& operator[](size_t i) { return polynomials_[i]; }
  const Polynomial& operator[](size_t i) const { return polynomials_[i]; }
  std::vector<double> evaluate(double t, int derivative) const {  // src/segment.cpp:51-58
    std::vector<double> out(D_);
    for (int d = 0; d < D_; ++d) out[d] = polynomials_[d].evaluate(t, derivative);
    return out;
  }

 private:
  int N_, D_;
  double time_ = 0.0;
  Polynomial::Vector polynomials_;
};

// ---------------------------------------------------------------------------- Trajectory
class Trajectory {
 public:
  int D() const { return segments_.empty() ? 0 : segments_.front().D(); }
  int N() const { return segments_.empty() ? 0 : segments_.front().N(); }
  int K() const { return (int)segments_.size(); }
  bool empty() const { return segments_.empty(); }
  void clear() { segments_.clear(); }
  void setSegments(const Segment::Vector& s) { segments_ = s; }
  void getSegments(Segment::Vector* s) const { *s = segments_; }
  const Segment::Vector& segments() const { return segments_; }
  double getMinTime() const { return 0.0; }
  double getMaxTime() const {
    double t = 0.0;
    for (const auto& s : segments_) t += s.getTime();
    return t;
  }
  std::vector<double> getSegmentTimes() const {
    std::vector<double> t;
    for (const auto& s : segments_) t.push_back(s.getTime());
    return t;
  }
  // Trajectory::evaluate (src/trajectory.cpp:41-66): the segment containing t (t beyond the end is
  // evaluated on the last segment, as the reference does)
  std::vector<double> evaluate(double t, int derivative = derivative_order::POSITION) const {
    double acc = 0.0;
    size_t i = 0;
    for (; i < segments_.size(); ++i) {
      acc += segments_[i].getTime();
      if (acc > t) break;
    }
    if (i >= segments_.size()) i = segments_.size() - 1;
    acc -= segments_[i].getTime();
    return segments_[i].evaluate(t - acc, derivative);
  }
  // Trajectory::evaluateRange (src/trajectory.cpp:68-128), on the GPU (mtg_evaluate_range_batch)
  void evaluateRange(double t_start, double t_end, double dt, int derivative, std::vector<std::vector<double>>* result,
                     std::vector<double>* sampling_times = nullptr) const {
    result->clear();
    if (sampling_times) sampling_times->clear();
    if (segments_.empty()) return;
    const int K = this->K(), D = this->D(), N = this->N();
    std::vector<double> coeffs((size_t)K * D * N), times(K);
    for (int i = 0; i < K; ++i) {
      times[i] = segments_[i].getTime();
      for (int d = 0; d < D; ++d) {
        const auto& c = segments_[i][d].getCoefficients();
        std::copy(c.begin(), c.end(), coeffs.begin() + ((size_t)i * D + d) * N);
      }
    }
    mtg_ctx* ctx = default_context();
    int64_t count = 0, offset = 0;
    check(mtg_evaluate_range_batch(ctx, N, D, K, 1, nullptr, times.data(), t_start, t_end, dt, derivative, &count,
                                   nullptr, nullptr, nullptr, 0),
          ctx, "mtg_evaluate_range_batch(count)");
    std::vector<double> out((size_t)std::max<int64_t>(count, 1) * D), st(std::max<int64_t>(count, 1));
    check(mtg_evaluate_range_batch(ctx, N, D, K, 1, coeffs.data(), times.data(), t_start, t_end, dt, derivative,
                                   &count, &offset, out.data(), st.data(), 0),
          ctx, "mtg_evaluate_range_batch");
    result->resize(count, std::vector<double>(D));
    for (int64_t s = 0; s < count; ++s)
      for (int d = 0; d < D; ++d) (*result)[s][d] = out[(size_t)s * D + d];
    if (sampling_times) sampling_times->assign(st.begin(), st.begin() + count);
  }

  // Trajectory::computeMinMaxMagnitude (src/trajectory.cpp:181-218), on the GPU
  // (mtg_min_max_magnitude_batch); Extremum as in the reference (extremum.h): segment-local time,
  // value, segment index
  struct Extremum {
    double time = 0.0, value = 0.0;
    int segment_idx = -1;
  };
  bool computeMinMaxMagnitude(int derivative, const std::vector<int>& dimensions, Extremum* minimum,
                              Extremum* maximum) const {
    if (segments_.empty() || dimensions.empty()) return false;
    const int K = this->K(), D = this->D(), N = this->N();
    std::vector<double> coeffs((size_t)K * D * N), times(K);
    for (int i = 0; i < K; ++i) {
      times[i] = segments_[i].getTime();
      for (int d = 0; d < D; ++d) {
        const auto& c = segments_[i][d].getCoefficients();
        std::copy(c.begin(), c.end(), coeffs.begin() + ((size_t)i * D + d) * N);
      }
    }
    uint32_t mask = 0;
    for (int d : dimensions) {
      if (d < 0 || d >= D) return false;  // segment.cpp:101-106: out-of-range dimension
      mask |= 1u << d;
    }
    mtg_ctx* ctx = default_context();
    mtg_extremum mn, mx;
    check(mtg_min_max_magnitude_batch(ctx, N, D, K, 1, coeffs.data(), times.data(), derivative, mask, &mn, &mx, 0),
          ctx, "mtg_min_max_magnitude_batch");
    *minimum = Extremum{mn.time, mn.value, mn.segment};
    *maximum = Extremum{mx.time, mx.value, mx.segment};
    return true;
  }

 private:
  Segment::Vector segments_;
};

// -------------------------------------------------------- packing Vertex::Vector -> ABI layout
// values [V][h][D] (fixed derivatives only), mask [V] (bit k: derivative k fixed; orders >= h are
// dropped with a warning, and flagged in bit 7 so the kernel reports MTG_TRAJ_WARN_DROPPED)
inline void pack_vertices(const Vertex::Vector& vertices, int N, int D, double* values, uint8_t* mask) {
  const int h = N / 2;
  const int V = (int)vertices.size();
  std::fill(values, values + (size_t)V * h * D, 0.0);
  for (int v = 0; v < V; ++v) {
    if (vertices[v].D() != D) fail(MTG_ERR_SIZE_MISMATCH, "vertex dimension mismatch");
    unsigned m = 0;
    for (auto it = vertices[v].cBegin(); it != vertices[v].cEnd(); ++it) {
      const int k = it->first;
      if (k < 0) fail(MTG_ERR_INVALID_ARGUMENT, "negative derivative order");
      if (k >= h) {
        std::fprintf(stderr,
                     "mtg: warning: invalid constraint of derivative order %d at vertex %d ignored "
                     "(max order N/2-1 = %d)\n", k, v, h - 1);
        m |= 0x80u;
        continue;
      }
      m |= 1u << k;
      for (int d = 0; d < D; ++d) values[((size_t)v * h + k) * D + d] = it->second[d];
    }
    mask[v] = (uint8_t)m;
  }
}

// ---------------------------------------------------------------- PolynomialOptimization<N>
template <int _N = 10>
class PolynomialOptimization {
  static_assert(_N % 2 == 0, "The number of coefficients has to be even.");
  static_assert(_N >= 2 && _N <= 12, "N must be in [2, 12]");

 public:
  enum { N = _N };
  static constexpr int kHighestDerivativeToOptimize = N / 2 - 1;

  explicit PolynomialOptimization(size_t dimension) : D_((int)dimension) {}

  // setupFromVertices (lin_impl:47-99)
  bool setupFromVertices(const Vertex::Vector& vertices, const std::vector<double>& segment_times,
                         int derivative_to_optimize = kHighestDerivativeToOptimize) {
    if (derivative_to_optimize < 0 || derivative_to_optimize > kHighestDerivativeToOptimize)
      fail(MTG_ERR_BAD_DERIVATIVE, "derivative_to_optimize out of [0, N/2-1]");
    if (vertices.size() != segment_times.size() + 1)
      fail(MTG_ERR_SIZE_MISMATCH, "vertices.size() must equal segment_times.size() + 1");
    r_ = derivative_to_optimize;
    K_ = (int)segment_times.size();
    vertices_ = vertices;
    values_.assign((size_t)(K_ + 1) * (N / 2) * D_, 0.0);
    mask_.assign(K_ + 1, 0);
    pack_vertices(vertices_, N, D_, values_.data(), mask_.data());
    updateSegmentTimes(segment_times);
    solved_ = false;
    return true;
  }

  // updateSegmentTimes (lin_impl:276-295)
  void updateSegmentTimes(const std::vector<double>& segment_times) {
    if ((int)segment_times.size() != K_) fail(MTG_ERR_SIZE_MISMATCH, "segment_times size mismatch");
    for (double t : segment_times)
      if (!(t > 0.0)) fail(MTG_ERR_INVALID_ARGUMENT, "segment times need to be greater than zero");
    times_ = segment_times;
    solved_ = false;
  }

  // solveLinear (lin_impl:329-369): one trajectory through the batched GPU solver
  bool solveLinear() {
    mtg_ctx* ctx = default_context();
    const int V = K_ + 1, h = N / 2;
    coeffs_.assign((size_t)K_ * D_ * N, 0.0);
    free_.assign((size_t)D_ * V * h, 0.0);
    int32_t nfree = 0, status = 0;
    check(mtg_solve_linear_batch(ctx, N, D_, K_, r_, 1, values_.data(), mask_.data(), times_.data(), coeffs_.data(),
                                 free_.data(), &nfree, &cost_, &status, 0),
          ctx, "mtg_solve_linear_batch");
    if (status & MTG_TRAJ_BAD_TIME) fail(MTG_ERR_INVALID_ARGUMENT, "segment times need to be greater than zero");
    n_free_ = nfree;
    solved_ = true;
    return true;
  }

  double computeCost() const { return cost_; }  // lin_impl:114-130 (0.5 sum c^T Q c)

  void getSegments(Segment::Vector* segments) const {
    segments->clear();
    for (int i = 0; i < K_; ++i) {
      Segment s(N, D_);
      s.setTime(times_[i]);
      for (int d = 0; d < D_; ++d) {
        const double* c = coeffs_.data() + ((size_t)i * D_ + d) * N;
        s[d] = Polynomial(std::vector<double>(c, c + N));
      }
      segments->push_back(std::move(s));
    }
  }
  void getTrajectory(Trajectory* trajectory) const {
    Segment::Vector s;
    getSegments(&s);
    trajectory->setSegments(s);
  }
  void getSegmentTimes(std::vector<double>* t) const { *t = times_; }
  void getVertices(Vertex::Vector* v) const { *v = vertices_; }
  // getFreeConstraints (polynomial_optimization_linear.h:180-184): per dimension, free
  // derivatives in (vertex, derivative) order
  void getFreeConstraints(std::vector<std::vector<double>>* free_constraints) const {
    const int V = K_ + 1, h = N / 2;
    free_constraints->assign(D_, std::vector<double>(n_free_));
    for (int d = 0; d < D_; ++d)
      for (int i = 0; i < n_free_; ++i) (*free_constraints)[d][i] = free_[(size_t)d * V * h + i];
  }
  // getFixedConstraints (polynomial_optimization_linear.h:188-192): per dimension, fixed
  // derivatives in (vertex, derivative) order
  void getFixedConstraints(std::vector<std::vector<double>>* fixed_constraints) const {
    const int V = K_ + 1, h = N / 2;
    fixed_constraints->assign(D_, std::vector<double>());
    for (int v = 0; v < V; ++v)
      for (int k = 0; k < h; ++k)
        if ((mask_[v] >> k) & 1u)
          for (int d = 0; d < D_; ++d) (*fixed_constraints)[d].push_back(values_[((size_t)v * h + k) * D_ + d]);
  }
  // setFreeConstraints (polynomial_optimization_linear.h:185-186) + updateSegmentsFromCompactConstraints
  // (lin_impl:253-273): new free derivatives (per dimension, reference order), coefficients recomputed
  // on the GPU (mtg_coefficients_from_vertices_batch); computeCost() follows the new coefficients.
  void setFreeConstraints(const std::vector<std::vector<double>>& free_constraints) {
    const int V = K_ + 1, h = N / 2;
    if ((int)free_constraints.size() != D_) fail(MTG_ERR_SIZE_MISMATCH, "setFreeConstraints: dimension mismatch");
    const int nf = (int)(V * h - getNumberFixedConstraints());
    std::vector<double> x((size_t)V * h * D_, 0.0);
    free_.assign((size_t)D_ * V * h, 0.0);
    for (int d = 0; d < D_; ++d) {
      if ((int)free_constraints[d].size() != nf) fail(MTG_ERR_SIZE_MISMATCH, "setFreeConstraints: size mismatch");
      int idx = 0;
      for (int v = 0; v < V; ++v)
        for (int k = 0; k < h; ++k) {
          const size_t o = ((size_t)v * h + k) * D_ + d;
          if ((mask_[v] >> k) & 1u) {
            x[o] = values_[o];
          } else {
            x[o] = free_constraints[d][idx];
            free_[(size_t)d * V * h + idx] = free_constraints[d][idx];
            ++idx;
          }
        }
    }
    n_free_ = nf;
    mtg_ctx* ctx = default_context();
    coeffs_.assign((size_t)K_ * D_ * N, 0.0);
    check(mtg_coefficients_from_vertices_batch(ctx, N, D_, K_, 1, x.data(), times_.data(), coeffs_.data(), 0), ctx,
          "mtg_coefficients_from_vertices_batch");
    std::vector<double> scales(K_, 1.0);
    double J = 0.0;
    check(mtg_cost_at_times_batch(ctx, N, D_, K_, r_, 1, x.data(), nullptr, times_.data(), 1, scales.data(), &J,
                                  nullptr, 0),
          ctx, "mtg_cost_at_times_batch");
    cost_ = 0.5 * J;  // computeCost = 0.5 sum c^T Q c; J = d^T R d (nl_impl:1499-1502)
    solved_ = true;
  }
  size_t getNumberFreeConstraints() const { return n_free_; }
  size_t getNumberFixedConstraints() const {
    size_t n = 0;
    for (uint8_t m : mask_) n += __builtin_popcount(m & ((1u << (N / 2)) - 1u));
    return n;
  }
  size_t getNumberAllConstraints() const { return getNumberFixedConstraints() + getNumberFreeConstraints(); }
  int getDimension() const { return D_; }
  int getDerivativeToOptimize() const { return r_; }

 private:
  int D_, K_ = 0, r_ = kHighestDerivativeToOptimize;
  bool solved_ = false;
  Vertex::Vector vertices_;
  std::vector<double> values_, times_, coeffs_, free_;
  std::vector<uint8_t> mask_;
  int n_free_ = 0;
  double cost_ = 0.0;
};

// PolynomialOptimizationNonLinear::computeInitialSolutionWithoutPositionConstraints
// (polynomial_optimization_nonlinear_impl.h:116-187) on a linear problem: solve, remove the position
// constraint of every interior vertex, set the problem up again with the same times and start its
// free derivatives from the solved trajectory (M^+ A p, mtg_vertex_derivatives_batch).  The
// polynomials are unchanged up to rounding; the free vector now holds the interior positions too.
template <int N>
bool computeInitialSolutionWithoutPositionConstraints(PolynomialOptimization<N>* opt) {
  opt->solveLinear();
  Segment::Vector segments;
  opt->getSegments(&segments);
  std::vector<double> times;
  opt->getSegmentTimes(&times);
  Vertex::Vector vertices;
  opt->getVertices(&vertices);
  const int K = (int)times.size(), D = opt->getDimension(), h = N / 2, V = K + 1;
  std::vector<double> coeffs((size_t)K * D * N), x((size_t)V * h * D);
  for (int i = 0; i < K; ++i)
    for (int d = 0; d < D; ++d) {
      const auto& c = segments[i][d].getCoefficients();
      for (int j = 0; j < N; ++j) coeffs[((size_t)i * D + d) * N + j] = c[j];
    }
  mtg_ctx* ctx = default_context();
  check(mtg_vertex_derivatives_batch(ctx, N, D, K, 1, coeffs.data(), times.data(), x.data(), 0), ctx,
        "mtg_vertex_derivatives_batch");
  for (int v = 1; v < V - 1; ++v) vertices[v].removeConstraint(derivative_order::POSITION);
  opt->setupFromVertices(vertices, times, opt->getDerivativeToOptimize());
  std::vector<std::vector<double>> free(D);
  for (int v = 0; v < V; ++v)
    for (int k = 0; k < h; ++k)
      if (!vertices[v].hasConstraint(k))
        for (int d = 0; d < D; ++d) free[d].push_back(x[((size_t)v * h + k) * D + d]);
  opt->setFreeConstraints(free);
  return true;
}

// ------------------------------------------------------------- BatchPolynomialOptimization<N>
// B independent problems of one shape (N, D, K, r) per call: the throughput API.  Arrays are in
// the ABI layout (mtg.h); pass MTG_FLAG_DEVICE_PTRS to hand over device pointers.
template <int _N = 10>
class BatchPolynomialOptimization {
 public:
  enum { N = _N };
  BatchPolynomialOptimization(int dimension, int segments, int derivative_to_optimize, int device = 0)
      : D_(dimension), K_(segments), r_(derivative_to_optimize) {
    check(mtg_create(device, &ctx_), nullptr, "mtg_create");
  }
  ~BatchPolynomialOptimization() { mtg_destroy(ctx_); }
  BatchPolynomialOptimization(const BatchPolynomialOptimization&) = delete;
  BatchPolynomialOptimization& operator=(const BatchPolynomialOptimization&) = delete;

  void solve(int64_t batch, const double* values, const uint8_t* mask, const double* times, double* coeffs,
             double* cost = nullptr, int32_t* status = nullptr, unsigned flags = 0) {
    check(mtg_solve_linear_batch(ctx_, N, D_, K_, r_, batch, values, mask, times, coeffs, nullptr, nullptr, cost,
                                 status, flags),
          ctx_, "mtg_solve_linear_batch");
  }
  void timeSweep(int64_t batch, const double* values, const uint8_t* mask, const double* times, int n_candidates,
                 const double* scales, double* cost, int32_t* status = nullptr, unsigned flags = 0) {
    check(mtg_time_sweep_batch(ctx_, N, D_, K_, r_, batch, values, mask, times, n_candidates, scales, cost, status,
                               flags),
          ctx_, "mtg_time_sweep_batch");
  }
  // config 5: cost sweep + segment-time Jacobian on the matrix cores (mtg_time_jacobian_batch)
  void timeJacobian(int64_t batch, const double* vertex_values, const double* times, int n_candidates,
                    const double* scales, double* cost, double* jac, double increment_time = 0.0,
                    unsigned flags = 0) {
    check(mtg_time_jacobian_batch(ctx_, N, D_, K_, r_, batch, vertex_values, times, n_candidates, scales,
                                  increment_time, cost, jac, flags),
          ctx_, "mtg_time_jacobian_batch");
  }
  void coefficientsFromVertices(int64_t batch, const double* vertex_values, const double* times, double* coeffs,
                                unsigned flags = 0) {
    check(mtg_coefficients_from_vertices_batch(ctx_, N, D_, K_, batch, vertex_values, times, coeffs, flags), ctx_,
          "mtg_coefficients_from_vertices_batch");
  }
  void vertexDerivatives(int64_t batch, const double* coeffs, const double* times, double* vertex_values,
                         unsigned flags = 0) {
    check(mtg_vertex_derivatives_batch(ctx_, N, D_, K_, batch, coeffs, times, vertex_values, flags), ctx_,
          "mtg_vertex_derivatives_batch");
  }
  void minMaxMagnitude(int64_t batch, const double* coeffs, const double* times, int derivative,
                       uint32_t dimension_mask, mtg_extremum* minimum, mtg_extremum* maximum, unsigned flags = 0) {
    check(mtg_min_max_magnitude_batch(ctx_, N, D_, K_, batch, coeffs, times, derivative, dimension_mask, minimum,
                                      maximum, flags),
          ctx_, "mtg_min_max_magnitude_batch");
  }
  mtg_ctx* context() const { return ctx_; }

 private:
  int D_, K_, r_;
  mtg_ctx* ctx_ = nullptr;
};

}  // namespace mtg
