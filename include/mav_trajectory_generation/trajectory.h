// trajectory.h -- Trajectory: a sequence of segments (reference trajectory.h:29-114,
// src/trajectory.cpp).
//
// evaluateRange keeps the reference's sequential clock (accumulated_time += dt, the strict '>'
// segment switch, sampling times restarting at the start segment's beginning), so its samples are
// bit-identical to the reference's.  A single trajectory is sampled on the calling thread (the
// library's GPU evaluateRange, mtg_evaluate_range_batch, is the batched form and gives the same
// bits); under ExecutionPolicy::kDevice it goes through the GPU.  computeMinMaxMagnitude follows the
// same policy (host: mtg_host_min_max_magnitude_batch; device: mtg_min_max_magnitude_batch).
#ifndef MAV_TRAJECTORY_GENERATION_TRAJECTORY_H_
#define MAV_TRAJECTORY_GENERATION_TRAJECTORY_H_

#include <algorithm>
#include <limits>
#include <vector>

#include "mav_trajectory_generation/extremum.h"
#include "mav_trajectory_generation/segment.h"

namespace mav_trajectory_generation {

class Trajectory {
 public:
  Trajectory() : D_(0), N_(0), max_time_(0.0) {}

  bool operator==(const Trajectory& rhs) const { return segments_ == rhs.segments_; }
  bool operator!=(const Trajectory& rhs) const { return !operator==(rhs); }

  int D() const { return D_; }
  int N() const { return N_; }
  int K() const { return (int)segments_.size(); }
  bool empty() const { return segments_.empty(); }
  void clear() {
    segments_.clear();
    D_ = 0;
    N_ = 0;
    max_time_ = 0.0;
  }

  void setSegments(const Segment::Vector& segments) {
    if (segments.empty()) fail(MTG_ERR_INVALID_ARGUMENT, "Trajectory::setSegments: no segments");
    segments_ = segments;
    D_ = segments_.front().D();
    N_ = segments_.front().N();
    max_time_ = 0.0;
    for (const Segment& segment : segments_) {
      if (segment.D() != D_) fail(MTG_ERR_SIZE_MISMATCH, "Trajectory::setSegments: dimension mismatch");
      max_time_ += segment.getTime();
    }
  }
  void getSegments(Segment::Vector* segments) const { *check_notnull(segments, "segments") = segments_; }
  const Segment::Vector& segments() const { return segments_; }

  double getMinTime() const { return 0.0; }
  double getMaxTime() const { return max_time_; }
  std::vector<double> getSegmentTimes() const {
    std::vector<double> t;
    t.reserve(segments_.size());
    for (const Segment& s : segments_) t.push_back(s.getTime());
    return t;
  }

  // src/trajectory.cpp:133-151
  Trajectory getTrajectoryWithSingleDimension(int dimension) const {
    if (dimension >= D_) fail(MTG_ERR_INVALID_ARGUMENT, "dimension out of range");
    Segment::Vector segments;
    segments.reserve(segments_.size());
    for (const Segment& s : segments_) {
      Segment segment(N_, 1);
      segment.setTime(s.getTime());
      segment[0] = s[dimension];
      segments.push_back(segment);
    }
    Trajectory traj;
    traj.setSegments(segments);
    return traj;
  }

  // src/trajectory.cpp:153-183
  Trajectory getTrajectoryWithAppendedDimension(const Trajectory& trajectory_to_append) const {
    if (N_ == 0 || D_ == 0) return trajectory_to_append;
    if (trajectory_to_append.N() == 0 || trajectory_to_append.D() == 0) return *this;
    if (N_ != trajectory_to_append.N() || K() != trajectory_to_append.K())
      fail(MTG_ERR_SIZE_MISMATCH, "getTrajectoryWithAppendedDimension: N and K must match");
    Segment::Vector segments;
    segments.reserve(segments_.size());
    for (size_t k = 0; k < segments_.size(); ++k) {
      Segment segment(N_, D_ + trajectory_to_append.D());
      segment.setTime(segments_[k].getTime());
      for (int d = 0; d < D_; ++d) segment[d] = segments_[k][d];
      for (int d = 0; d < trajectory_to_append.D(); ++d) segment[D_ + d] = trajectory_to_append.segments()[k][d];
      segments.push_back(segment);
    }
    Trajectory traj;
    traj.setSegments(segments);
    return traj;
  }

  // src/trajectory.cpp:41-66: the segment whose accumulated end time first exceeds t.  Beyond the
  // end the reference logs an error and returns zeros; at exactly the end time (where the
  // reference indexes one past the last segment) the last segment is evaluated at its end.
  VectorXd evaluate(double t, int derivative_order = derivative_order::POSITION) const {
    double accumulated_time = 0.0;
    size_t i = 0;
    for (i = 0; i < segments_.size(); ++i) {
      accumulated_time += segments_[i].getTime();
      if (accumulated_time > t) break;
    }
    if (t > accumulated_time || segments_.empty()) {
      std::fprintf(stderr, "mav_trajectory_generation: error: Time out of range of the trajectory!\n");
      return VectorXd::Zero(D_);
    }
    if (i == segments_.size()) i = segments_.size() - 1;
    accumulated_time -= segments_[i].getTime();
    return segments_[i].evaluate(t - accumulated_time, derivative_order);
  }

  // src/trajectory.cpp:68-128
  void evaluateRange(double t_start, double t_end, double dt, int derivative_order, std::vector<VectorXd>* result,
                     std::vector<double>* sampling_times = nullptr) const {
    check_notnull(result, "result");
    result->clear();
    if (sampling_times) sampling_times->clear();
    if (segments_.empty()) return;
    if (singleOnDevice()) {
      evaluateRangeDevice(t_start, t_end, dt, derivative_order, result, sampling_times);
      return;
    }
    const size_t expected = (size_t)std::max(0.0, (t_end - t_start) / dt + 1);
    result->reserve(expected);
    if (sampling_times) sampling_times->reserve(expected);
    double accumulated_time = 0.0;
    size_t i = 0;
    for (i = 0; i < segments_.size(); ++i) {
      accumulated_time += segments_[i].getTime();
      if (accumulated_time > t_start) break;
    }
    if (t_start > accumulated_time || i == segments_.size()) {
      std::fprintf(stderr, "mav_trajectory_generation: error: Start time out of range of the trajectory!\n");
      return;
    }
    accumulated_time -= segments_[i].getTime();
    double time_in_segment = t_start - accumulated_time;
    while (accumulated_time < t_end) {
      if (time_in_segment > segments_[i].getTime()) {
        time_in_segment = time_in_segment - segments_[i].getTime();
        i++;
        if (i >= segments_.size()) break;
        continue;
      }
      result->push_back(segments_[i].evaluate(time_in_segment, derivative_order));
      if (sampling_times) sampling_times->push_back(accumulated_time);
      time_in_segment += dt;
      accumulated_time += dt;
    }
  }

  // The same samples through the GPU kernels (mtg_evaluate_range_batch, one trajectory).
  void evaluateRangeDevice(double t_start, double t_end, double dt, int derivative_order,
                           std::vector<VectorXd>* result, std::vector<double>* sampling_times = nullptr) const {
    check_notnull(result, "result");
    result->clear();
    if (sampling_times) sampling_times->clear();
    if (segments_.empty()) return;
    std::vector<double> coeffs, times;
    pack(&coeffs, &times);
    mtg_ctx* ctx = defaultContext();
    int64_t count = 0, offset = 0;
    check(mtg_evaluate_range_batch(ctx, N_, D_, K(), 1, nullptr, times.data(), t_start, t_end, dt, derivative_order,
                                   &count, nullptr, nullptr, nullptr, 0),
          ctx, "mtg_evaluate_range_batch(count)");
    std::vector<double> out((size_t)std::max<int64_t>(count, 1) * D_), st((size_t)std::max<int64_t>(count, 1));
    check(mtg_evaluate_range_batch(ctx, N_, D_, K(), 1, coeffs.data(), times.data(), t_start, t_end, dt,
                                   derivative_order, &count, &offset, out.data(), st.data(), 0),
          ctx, "mtg_evaluate_range_batch");
    result->reserve((size_t)count);
    for (int64_t s = 0; s < count; ++s) {
      VectorXd v(D_);
      for (int d = 0; d < D_; ++d) v[d] = out[(size_t)s * D_ + d];
      result->push_back(v);
    }
    if (sampling_times) sampling_times->assign(st.begin(), st.begin() + count);
  }

  // src/trajectory.cpp:185-218: per segment the candidates t = 0, t = T and the real roots in [0, T]
  // of the magnitude's derivative; segment-local times.  On the host (mtg_host_min_max_magnitude_batch)
  // unless ExecutionPolicy::kDevice, which runs the GPU kernel (mtg_min_max_magnitude_batch).
  bool computeMinMaxMagnitude(int derivative, const std::vector<int>& dimensions, Extremum* minimum,
                              Extremum* maximum) const {
    check_notnull(minimum, "minimum");
    check_notnull(maximum, "maximum");
    minimum->value = std::numeric_limits<double>::max();
    maximum->value = std::numeric_limits<double>::lowest();
    if (segments_.empty() || dimensions.empty()) return false;
    uint32_t mask = 0;
    for (int d : dimensions) {
      if (d < 0 || d >= D_ || d >= 32) return false;  // src/segment.cpp:101-106
      mask |= 1u << d;
    }
    std::vector<double> coeffs, times;
    pack(&coeffs, &times);
    mtg_extremum mn, mx;
    if (singleOnDevice()) {
      mtg_ctx* ctx = defaultContext();
      check(mtg_min_max_magnitude_batch(ctx, N_, D_, K(), 1, coeffs.data(), times.data(), derivative, mask, &mn, &mx,
                                        0),
            ctx, "mtg_min_max_magnitude_batch");
    } else {  // the reference computes this on the CPU too
      check(mtg_host_min_max_magnitude_batch(N_, D_, K(), 1, coeffs.data(), times.data(), derivative, mask, &mn, &mx,
                                             1),
            nullptr, "mtg_host_min_max_magnitude_batch");
    }
    *minimum = Extremum(mn.time, mn.value, mn.segment);
    *maximum = Extremum(mx.time, mx.value, mx.segment);
    return true;
  }

  // coefficients [K][D][N] and times [K] in the C ABI layout
  void pack(std::vector<double>* coeffs, std::vector<double>* times) const {
    coeffs->assign((size_t)K() * D_ * N_, 0.0);
    times->assign((size_t)K(), 0.0);
    for (int i = 0; i < K(); ++i) {
      (*times)[i] = segments_[i].getTime();
      for (int d = 0; d < D_; ++d) {
        const VectorXd c = segments_[i][d].getCoefficients();
        for (int j = 0; j < N_; ++j) (*coeffs)[((size_t)i * D_ + d) * N_ + j] = c[j];
      }
    }
  }

 private:
  int D_;
  int N_;
  double max_time_;
  Segment::Vector segments_;
};

}  // namespace mav_trajectory_generation

#endif  // MAV_TRAJECTORY_GENERATION_TRAJECTORY_H_
