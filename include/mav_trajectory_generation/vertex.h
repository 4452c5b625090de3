// vertex.h -- Vertex and the vertex helpers (reference vertex.h:33-149, src/vertex.cpp).
//
// A Vertex holds, per derivative order, a D-vector of fixed values.  The generators are the
// library's (mtg_host_random_vertices_batch, mtg_host_estimate_segment_times): std::mt19937 +
// uniform_real_distribution and Eigen's norm reduction order, so vertices and times are
// bit-identical to the reference's on x86-64.
#ifndef MAV_TRAJECTORY_GENERATION_VERTEX_H_
#define MAV_TRAJECTORY_GENERATION_VERTEX_H_

#include <map>
#include <ostream>
#include <utility>
#include <vector>

#include "mav_trajectory_generation/linalg.h"
#include "mav_trajectory_generation/motion_defines.h"
#include "mav_trajectory_generation/runtime.h"

namespace mav_trajectory_generation {

class Vertex {
 public:
  typedef std::vector<Vertex> Vector;
  typedef VectorXd ConstraintValue;
  typedef std::pair<int, ConstraintValue> Constraint;
  typedef std::map<int, ConstraintValue> Constraints;

  explicit Vertex(size_t dimension) : D_((int)dimension) {}

  int D() const { return D_; }

  void addConstraint(int derivative_order, double value) {
    constraints_[derivative_order] = ConstraintValue::Constant(D_, value);
  }
  void addConstraint(int type, const VectorXd& constraint) {  // src/vertex.cpp:86-90
    if ((int)constraint.rows() != D_) fail(MTG_ERR_SIZE_MISMATCH, "Vertex::addConstraint: dimension mismatch");
    constraints_[type] = constraint;
  }
  bool removeConstraint(int type) { return constraints_.erase(type) > 0; }

  void makeStartOrEnd(const VectorXd& constraint, int up_to_derivative) {  // src/vertex.cpp:104-110
    addConstraint(derivative_order::POSITION, constraint);
    for (int i = 1; i <= up_to_derivative; ++i) constraints_[i] = ConstraintValue::Zero(D_);
  }
  void makeStartOrEnd(double value, int up_to_derivative) {
    makeStartOrEnd(ConstraintValue::Constant(D_, value), up_to_derivative);
  }

  bool hasConstraint(int derivative_order) const { return constraints_.count(derivative_order) > 0; }
  bool getConstraint(int derivative_order, VectorXd* constraint) const {
    check_notnull(constraint, "constraint");
    auto it = constraints_.find(derivative_order);
    if (it == constraints_.end()) return false;
    *constraint = it->second;
    return true;
  }

  Constraints::const_iterator cBegin() const { return constraints_.begin(); }
  Constraints::const_iterator cEnd() const { return constraints_.end(); }
  size_t getNumberOfConstraints() const { return constraints_.size(); }

  bool isEqualTol(const Vertex& rhs, double tol) const {  // src/vertex.cpp:130-145
    if (constraints_.size() != rhs.constraints_.size()) return false;
    for (const auto& c : constraints_) {
      auto it = rhs.constraints_.find(c.first);
      if (it == rhs.constraints_.end()) return false;
      if (!(c.second - it->second).isZero(tol)) return false;
    }
    return true;
  }

 private:
  int D_;
  Constraints constraints_;
};

inline std::ostream& operator<<(std::ostream& stream, const Vertex& v) {
  stream << "constraints: " << std::endl;
  for (auto it = v.cBegin(); it != v.cEnd(); ++it) {
    stream << "  type: " << positionDerivativeToString(it->first) << "  value: [";
    for (int d = 0; d < (int)it->second.size(); ++d) stream << (d ? ", " : "") << it->second[d];
    stream << "]" << std::endl;
  }
  return stream;
}

inline std::ostream& operator<<(std::ostream& stream, const std::vector<Vertex>& vertices) {
  for (const Vertex& v : vertices) stream << v << std::endl;
  return stream;
}

// t = 2 d / v_max (1 + magic v_max / a_max exp(-2 d / v_max)), d the distance between consecutive
// vertex positions (src/vertex.cpp:162-178).
inline std::vector<double> estimateSegmentTimes(const Vertex::Vector& vertices, double v_max, double a_max,
                                                double magic_fabian_constant = 6.5) {
  if (vertices.size() < 2) return {};
  const int D = vertices.front().D(), V = (int)vertices.size();
  std::vector<double> pos((size_t)V * D, 0.0), times(V - 1);
  for (int v = 0; v < V; ++v) {
    VectorXd p;
    if (vertices[v].getConstraint(derivative_order::POSITION, &p))
      for (int d = 0; d < D; ++d) pos[(size_t)v * D + d] = p[d];
  }
  check(mtg_host_estimate_segment_times(V, D, pos.data(), v_max, a_max, magic_fabian_constant, times.data()),
        nullptr, "mtg_host_estimate_segment_times");
  return times;
}

// Random positions in [minimum_position, maximum_position], consecutive vertices > 0.2 apart; the
// first and last vertex fix derivatives 0..maximum_derivative (zero above the position), the
// others only the position (src/vertex.cpp:27-79).
inline Vertex::Vector createRandomVertices(int maximum_derivative, size_t n_segments,
                                           const VectorXd& minimum_position, const VectorXd& maximum_position,
                                           size_t seed = 0) {
  if ((int)n_segments < 1) fail(MTG_ERR_SIZE_MISMATCH, "createRandomVertices: n_segments must be >= 1");
  if (minimum_position.size() != maximum_position.size())
    fail(MTG_ERR_SIZE_MISMATCH, "createRandomVertices: position bounds differ in size");
  if (maximum_derivative <= 0) fail(MTG_ERR_INVALID_ARGUMENT, "createRandomVertices: maximum_derivative must be > 0");
  const int D = (int)minimum_position.size(), K = (int)n_segments, V = K + 1;
  std::vector<double> pmin(D), pmax(D), values((size_t)V * D), times(K);
  std::vector<uint8_t> mask(V);
  for (int d = 0; d < D; ++d) pmin[d] = minimum_position[d], pmax[d] = maximum_position[d];
  // N = 2 packs only the positions; the generator draws them exactly as the reference does
  check(mtg_host_random_vertices_batch(2, D, K, maximum_derivative, pmin.data(), pmax.data(), (uint32_t)seed, 1, 1.0,
                                       1.0, 6.5, values.data(), mask.data(), times.data(), 1),
        nullptr, "mtg_host_random_vertices_batch");
  Vertex::Vector vertices(V, Vertex(D));
  for (int v = 0; v < V; ++v) {
    VectorXd p(D);
    for (int d = 0; d < D; ++d) p[d] = values[(size_t)v * D + d];
    if (v == 0 || v == K)
      vertices[v].makeStartOrEnd(p, maximum_derivative);
    else
      vertices[v].addConstraint(derivative_order::POSITION, p);
  }
  return vertices;
}

inline Vertex::Vector createRandomVertices1D(int maximum_derivative, size_t n_segments, double minimum_position,
                                             double maximum_position, size_t seed = 0) {
  return createRandomVertices(maximum_derivative, n_segments, VectorXd::Constant(1, minimum_position),
                              VectorXd::Constant(1, maximum_position), seed);
}

}  // namespace mav_trajectory_generation

#endif  // MAV_TRAJECTORY_GENERATION_VERTEX_H_
