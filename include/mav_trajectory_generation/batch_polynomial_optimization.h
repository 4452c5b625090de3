// batch_polynomial_optimization.h -- BatchPolynomialOptimization<N>: B independent problems of one
// shape (N, D, K, r) per call, on the GPU.  This is the throughput API the library exists for
// (BASELINE configs 2-5); the reference has no batched form -- its callers loop over
// PolynomialOptimization<N> (src/polynomial_timing_evaluation.cpp:119-126).
//
// Arrays are in the C ABI layout (include/mtg.h): values [B][K+1][N/2][D], mask [B][K+1] (bit k:
// derivative k fixed), times [B][K], coeffs [B][K][D][N].  Pass MTG_FLAG_DEVICE_PTRS to hand over
// device pointers (inputs already in HBM); host pointers are staged by the library.
//
// Several devices: construct with a device list (e.g. allDevices()).  A host-array solve() is then
// one mtg_solve_linear_batch_multi call: contiguous shards of the batch, one host thread and one
// context per device, no collective; bit-identical to a one-device solve.  Device-
// pointer calls and the other entry points run on the first device.
#ifndef MAV_TRAJECTORY_GENERATION_BATCH_POLYNOMIAL_OPTIMIZATION_H_
#define MAV_TRAJECTORY_GENERATION_BATCH_POLYNOMIAL_OPTIMIZATION_H_

#include <cstdint>
#include <vector>

#include "mav_trajectory_generation/runtime.h"
#include "mav_trajectory_generation/vertex.h"

namespace mav_trajectory_generation {

// Pack one Vertex::Vector into the ABI layout: values [V][h][D] (fixed derivatives), mask [V];
// orders >= h are dropped with a warning and flagged in bit 7 (the solver then reports
// MTG_TRAJ_WARN_DROPPED), as setupFromVertices does (lin_impl:74-95).
inline void packVertices(const Vertex::Vector& vertices, int N, int D, double* values, uint8_t* mask) {
  const int h = N / 2;
  const int V = (int)vertices.size();
  for (size_t i = 0; i < (size_t)V * h * D; ++i) values[i] = 0.0;
  for (int v = 0; v < V; ++v) {
    if (vertices[v].D() != D) fail(MTG_ERR_SIZE_MISMATCH, "vertex dimension mismatch");
    unsigned m = 0;
    for (auto it = vertices[v].cBegin(); it != vertices[v].cEnd(); ++it) {
      const int k = it->first;
      if (k < 0) continue;
      if (k >= h) {
        m |= 0x80u;
        continue;
      }
      m |= 1u << k;
      for (int d = 0; d < D; ++d) values[((size_t)v * h + k) * D + d] = it->second[d];
    }
    mask[v] = (uint8_t)m;
  }
}

template <int _N = 10>
class BatchPolynomialOptimization {
  static_assert(_N % 2 == 0 && _N >= 2 && _N <= 12, "N must be even and in [2, 12]");

 public:
  enum { N = _N };
  BatchPolynomialOptimization(int dimension, int segments, int derivative_to_optimize, int device = 0)
      : BatchPolynomialOptimization(dimension, segments, derivative_to_optimize, std::vector<int>{device}) {}
  BatchPolynomialOptimization(int dimension, int segments, int derivative_to_optimize, const std::vector<int>& devices)
      : D_(dimension), K_(segments), r_(derivative_to_optimize) {
    if (devices.empty()) fail(MTG_ERR_INVALID_ARGUMENT, "BatchPolynomialOptimization: no device");
    for (int device : devices) {
      mtg_ctx* c = nullptr;
      const int rc = mtg_create(device, &c);
      if (rc != MTG_OK) {
        for (mtg_ctx* o : ctxs_) mtg_destroy(o);
        ctxs_.clear();
        check(rc, nullptr, "mtg_create");
      }
      ctxs_.push_back(c);
    }
    ctx_ = ctxs_.front();
  }
  ~BatchPolynomialOptimization() {
    for (mtg_ctx* c : ctxs_) mtg_destroy(c);
  }
  // every visible device: 0 .. mtg_device_count() - 1
  static std::vector<int> allDevices() {
    int n = 0;
    check(mtg_device_count(&n), nullptr, "mtg_device_count");
    std::vector<int> d(n);
    for (int i = 0; i < n; ++i) d[i] = i;
    return d;
  }
  int numDevices() const { return (int)ctxs_.size(); }
  BatchPolynomialOptimization(const BatchPolynomialOptimization&) = delete;
  BatchPolynomialOptimization& operator=(const BatchPolynomialOptimization&) = delete;

  int dimension() const { return D_; }
  int segments() const { return K_; }
  int derivativeToOptimize() const { return r_; }
  mtg_ctx* context() const { return ctx_; }

  // setupFromVertices + solveLinear + getSegments / computeCost per problem (mtg_solve_linear_batch)
  void solve(int64_t batch, const double* values, const uint8_t* mask, const double* times, double* coeffs,
             double* cost = nullptr, int32_t* status = nullptr, unsigned flags = 0, double* free_out = nullptr,
             int32_t* n_free = nullptr) {
    if (ctxs_.size() > 1 && !(flags & (MTG_FLAG_DEVICE_PTRS | MTG_FLAG_ASYNC))) {
      check(mtg_solve_linear_batch_multi(ctxs_.data(), (int)ctxs_.size(), N, D_, K_, r_, batch, values, mask, times,
                                         coeffs, free_out, n_free, cost, status, flags),
            ctx_, "mtg_solve_linear_batch_multi");
      return;
    }
    check(mtg_solve_linear_batch(ctx_, N, D_, K_, r_, batch, values, mask, times, coeffs, free_out, n_free, cost,
                                 status, flags),
          ctx_, "mtg_solve_linear_batch");
  }
  // Problems given as Vertex lists (one per problem, all with K + 1 vertices) and segment times.
  void solve(const std::vector<Vertex::Vector>& problems, const std::vector<std::vector<double>>& times,
             std::vector<double>* coeffs, std::vector<double>* cost = nullptr, std::vector<int32_t>* status = nullptr) {
    const int64_t B = (int64_t)problems.size();
    const int V = K_ + 1, h = N / 2;
    if ((int64_t)times.size() != B) fail(MTG_ERR_SIZE_MISMATCH, "one segment-time vector per problem");
    std::vector<double> vals((size_t)B * V * h * D_), t((size_t)B * K_);
    std::vector<uint8_t> mask((size_t)B * V);
    for (int64_t b = 0; b < B; ++b) {
      if ((int)problems[b].size() != V || (int)times[b].size() != K_)
        fail(MTG_ERR_SIZE_MISMATCH, "every problem needs K + 1 vertices and K segment times");
      packVertices(problems[b], N, D_, vals.data() + (size_t)b * V * h * D_, mask.data() + (size_t)b * V);
      for (int i = 0; i < K_; ++i) t[(size_t)b * K_ + i] = times[b][i];
    }
    check_notnull(coeffs, "coeffs")->assign((size_t)B * K_ * D_ * N, 0.0);
    if (cost) cost->assign((size_t)B, 0.0);
    if (status) status->assign((size_t)B, 0);
    solve(B, vals.data(), mask.data(), t.data(), coeffs->data(), cost ? cost->data() : nullptr,
          status ? status->data() : nullptr);
  }
  // time-allocation sweep: optimal cost at scale[c] * times (mtg_time_sweep_batch)
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
  // cost (and gradient) of fixed vertex derivatives at candidate times (mtg_cost_at_times_batch)
  void costAtTimes(int64_t batch, const double* vertex_values, const uint8_t* mask, const double* times,
                   int n_candidates, const double* scales, double* cost, double* grad = nullptr, unsigned flags = 0) {
    check(mtg_cost_at_times_batch(ctx_, N, D_, K_, r_, batch, vertex_values, mask, times, n_candidates, scales, cost,
                                  grad, flags),
          ctx_, "mtg_cost_at_times_batch");
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
  // Trajectory::evaluateRange over the batch (mtg_evaluate_range_batch): counts [B]; then samples
  // [sum counts][D] (+ sampling times) at offsets (exclusive prefix sum of counts).
  void evaluateRangeCounts(int64_t batch, const double* times, double t_start, double t_end, double dt,
                           int64_t* counts, unsigned flags = 0) {
    check(mtg_evaluate_range_batch(ctx_, N, D_, K_, batch, nullptr, times, t_start, t_end, dt, 0, counts, nullptr,
                                   nullptr, nullptr, flags),
          ctx_, "mtg_evaluate_range_batch(count)");
  }
  void evaluateRange(int64_t batch, const double* coeffs, const double* times, double t_start, double t_end,
                     double dt, int derivative, int64_t* counts, const int64_t* offsets, double* out,
                     double* sampling_times = nullptr, unsigned flags = 0) {
    check(mtg_evaluate_range_batch(ctx_, N, D_, K_, batch, coeffs, times, t_start, t_end, dt, derivative, counts,
                                   offsets, out, sampling_times, flags),
          ctx_, "mtg_evaluate_range_batch");
  }

 private:
  int D_, K_, r_;
  std::vector<mtg_ctx*> ctxs_;
  mtg_ctx* ctx_ = nullptr;
};

}  // namespace mav_trajectory_generation

#endif  // MAV_TRAJECTORY_GENERATION_BATCH_POLYNOMIAL_OPTIMIZATION_H_
