// extremum.h -- Extremum (reference extremum.h:28-52).
//
// The struct, its comparison operators and its operator<< format restate the reference's public
// interface (mav_trajectory_generation/include/mav_trajectory_generation/extremum.h, Copyright (c)
// 2016 Markus Achtelik, Michael Burri, Helen Oleynikova, Rik Baehnemann, Marija Popovic, ASL, ETH
// Zurich; Apache License 2.0, http://www.apache.org/licenses/LICENSE-2.0): the names,
// fields and output format are the drop-in's contract.
#ifndef MAV_TRAJECTORY_GENERATION_EXTREMUM_H_
#define MAV_TRAJECTORY_GENERATION_EXTREMUM_H_

#include <ostream>

namespace mav_trajectory_generation {

// Time (relative to the segment start), value and segment of an extremum.
struct Extremum {
 public:
  Extremum() : time(0.0), value(0.0), segment_idx(0) {}
  Extremum(double _time, double _value, int _segment_idx) : time(_time), value(_value), segment_idx(_segment_idx) {}

  bool operator<(const Extremum& rhs) const { return value < rhs.value; }
  bool operator>(const Extremum& rhs) const { return value > rhs.value; }

  double time;
  double value;
  int segment_idx;
};

inline std::ostream& operator<<(std::ostream& stream, const Extremum& e) {
  stream << "time: " << e.time << ", value: " << e.value << ", segment idx: " << e.segment_idx << std::endl;
  return stream;
}

}  // namespace mav_trajectory_generation

#endif  // MAV_TRAJECTORY_GENERATION_EXTREMUM_H_
