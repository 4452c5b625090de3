// motion_defines.h -- derivative-order names (reference motion_defines.h:27-45, src/motion_defines.cpp).
#ifndef MAV_TRAJECTORY_GENERATION_MOTION_DEFINES_H_
#define MAV_TRAJECTORY_GENERATION_MOTION_DEFINES_H_

#include <string>

namespace mav_trajectory_generation {

namespace derivative_order {
static constexpr int POSITION = 0;
static constexpr int VELOCITY = 1;
static constexpr int ACCELERATION = 2;
static constexpr int JERK = 3;
static constexpr int SNAP = 4;

static constexpr int ORIENTATION = 0;
static constexpr int ANGULAR_VELOCITY = 1;
static constexpr int ANGULAR_ACCELERATION = 2;

static constexpr int kINVALID = -1;
}  // namespace derivative_order

inline std::string positionDerivativeToString(int derivative) {
  static const char* const kNames[] = {"position", "velocity", "acceleration", "jerk", "snap"};
  if (derivative >= 0 && derivative <= derivative_order::SNAP) return kNames[derivative];
  return "invalid";
}

inline int positionDerivativeToInt(const std::string& string) {
  for (int d = 0; d <= derivative_order::SNAP; ++d)
    if (string == positionDerivativeToString(d)) return d;
  return derivative_order::kINVALID;
}

inline std::string orintationDerivativeToString(int derivative) {  // (sic, reference spelling)
  static const char* const kNames[] = {"orientation", "angular_velocity", "angular_acceleration"};
  if (derivative >= 0 && derivative <= derivative_order::ANGULAR_ACCELERATION) return kNames[derivative];
  return "invalid";
}

inline int orientationDerivativeToInt(const std::string& string) {
  for (int d = 0; d <= derivative_order::ANGULAR_ACCELERATION; ++d)
    if (string == orintationDerivativeToString(d)) return d;
  return derivative_order::kINVALID;
}

}  // namespace mav_trajectory_generation

#endif  // MAV_TRAJECTORY_GENERATION_MOTION_DEFINES_H_
