// segment.h -- Segment: a time and one Polynomial per dimension (reference segment.h:37-131,
// src/segment.cpp:27-58).
//
// Not provided: computeMinMaxMagnitudeCandidate{Times,s} / selectMinMaxMagnitudeFromCandidates
// (root finding, src/rpoly.cpp); use Trajectory::computeMinMaxMagnitude (host or GPU, ExecutionPolicy).
#ifndef MAV_TRAJECTORY_GENERATION_SEGMENT_H_
#define MAV_TRAJECTORY_GENERATION_SEGMENT_H_

#include <cstdint>
#include <ostream>
#include <vector>

#include "mav_trajectory_generation/extremum.h"
#include "mav_trajectory_generation/motion_defines.h"
#include "mav_trajectory_generation/polynomial.h"

namespace mav_trajectory_generation {

constexpr double kNumNSecPerSec = 1.0e9;
constexpr double kNumSecPerNsec = 1.0e-9;

class Segment {
 public:
  typedef std::vector<Segment> Vector;

  Segment(int N, int D) : time_(0.0), N_(N), D_(D) { polynomials_.resize(D_, Polynomial(N_)); }
  Segment(const Segment& segment) = default;
  Segment& operator=(const Segment& segment) = default;

  bool operator==(const Segment& rhs) const {  // src/segment.cpp:27-40
    if (D_ != rhs.D_ || time_ != rhs.time_) return false;
    for (int i = 0; i < D_; ++i)
      if (polynomials_[i] != rhs.polynomials_[i]) return false;
    return true;
  }
  bool operator!=(const Segment& rhs) const { return !operator==(rhs); }

  int D() const { return D_; }
  int N() const { return N_; }
  double getTime() const { return time_; }
  uint64_t getTimeNSec() const { return static_cast<uint64_t>(kNumNSecPerSec * time_); }
  void setTime(double time_sec) { time_ = time_sec; }
  void setTimeNSec(uint64_t time_ns) { time_ = time_ns * kNumSecPerNsec; }

  Polynomial& operator[](size_t idx) {
    if (idx >= (size_t)D_) fail(MTG_ERR_INVALID_ARGUMENT, "Segment: dimension index out of range");
    return polynomials_[idx];
  }
  const Polynomial& operator[](size_t idx) const {
    if (idx >= (size_t)D_) fail(MTG_ERR_INVALID_ARGUMENT, "Segment: dimension index out of range");
    return polynomials_[idx];
  }
  const Polynomial::Vector& getPolynomialsRef() const { return polynomials_; }

  // src/segment.cpp:51-58
  VectorXd evaluate(double t, int derivative_order = derivative_order::POSITION) const {
    VectorXd result(D_);
    for (int d = 0; d < D_; ++d) result[d] = polynomials_[d].evaluate(t, derivative_order);
    return result;
  }

 protected:
  Polynomial::Vector polynomials_;
  double time_;

 private:
  int N_;
  int D_;
};

// printSegment (src/segment.cpp:60-80): time, then each dimension's coefficients.
inline void printSegment(std::ostream& stream, const Segment& s, int derivative) {
  stream << "t: " << s.getTime() << std::endl;
  stream << " coefficients for " << positionDerivativeToString(derivative) << ": " << std::endl;
  for (int i = 0; i < s.D(); ++i) {
    stream << "dim " << i << ": " << std::endl;
    const VectorXd c = s[i].getCoefficients(derivative);
    for (int j = 0; j < (int)c.size(); ++j) stream << (j ? " " : "") << c[j];
    stream << std::endl;
  }
}

inline std::ostream& operator<<(std::ostream& stream, const Segment& s) {
  printSegment(stream, s, derivative_order::POSITION);
  return stream;
}

inline std::ostream& operator<<(std::ostream& stream, const std::vector<Segment>& segments) {
  for (const Segment& s : segments) stream << s << std::endl;
  return stream;
}

}  // namespace mav_trajectory_generation

#endif  // MAV_TRAJECTORY_GENERATION_SEGMENT_H_
