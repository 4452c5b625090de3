// linalg.h -- the vector / matrix types of the drop-in API.
//
// The reference's public types are Eigen's (Eigen::VectorXd for constraint values and
// coefficients, Eigen::MatrixXd for getA/getM/getR/..., vertex.h:45, polynomial.h:52,
// polynomial_optimization_linear.h:209-214).  This image has no Eigen, so by default the drop-in
// uses the two small dense types below, which implement the subset of Eigen's interface the
// reference API and its callers use (size/rows/cols, operator()/[], Zero/Constant, setZero,
// resize, head/tail, norm, +, -, *, transpose, data()).  A project that has Eigen defines
// MTG_USE_EIGEN before including any header of this directory; the types are then Eigen's own.
// (The MTG_USE_EIGEN path cannot be compiled in this image; INTEGRATION.md.)
#ifndef MAV_TRAJECTORY_GENERATION_LINALG_H_
#define MAV_TRAJECTORY_GENERATION_LINALG_H_

#ifdef MTG_USE_EIGEN
#include <Eigen/Core>

namespace mav_trajectory_generation {
typedef Eigen::VectorXd VectorXd;
typedef Eigen::MatrixXd MatrixXd;
template <int R, int C>
using FixedMatrix = Eigen::Matrix<double, R, C>;
}  // namespace mav_trajectory_generation

#else
#include <cmath>
#include <cstddef>
#include <initializer_list>
#include <ostream>
#include <vector>

namespace mav_trajectory_generation {

typedef std::ptrdiff_t Index;

// Dense column vector of doubles (Eigen::VectorXd subset).  New storage is zero-initialised.
class VectorXd {
 public:
  VectorXd() = default;
  explicit VectorXd(Index n) : v_((size_t)n, 0.0) {}
  VectorXd(std::initializer_list<double> l) : v_(l) {}
  explicit VectorXd(const std::vector<double>& v) : v_(v) {}

  static VectorXd Zero(Index n) { return VectorXd(n); }
  static VectorXd Constant(Index n, double value) {
    VectorXd r(n);
    r.setConstant(value);
    return r;
  }

  Index size() const { return (Index)v_.size(); }
  Index rows() const { return size(); }
  Index cols() const { return 1; }
  double& operator[](Index i) { return v_[(size_t)i]; }
  double operator[](Index i) const { return v_[(size_t)i]; }
  double& operator()(Index i) { return v_[(size_t)i]; }
  double operator()(Index i) const { return v_[(size_t)i]; }
  double* data() { return v_.data(); }
  const double* data() const { return v_.data(); }

  void resize(Index n) { v_.assign((size_t)n, 0.0); }
  VectorXd& setZero() { return setConstant(0.0); }
  VectorXd& setConstant(double value) {
    for (double& x : v_) x = value;
    return *this;
  }
  VectorXd head(Index n) const { return VectorXd(std::vector<double>(v_.begin(), v_.begin() + n)); }
  VectorXd tail(Index n) const { return VectorXd(std::vector<double>(v_.end() - n, v_.end())); }
  VectorXd reverse() const { return VectorXd(std::vector<double>(v_.rbegin(), v_.rend())); }
  double squaredNorm() const {
    double s = 0.0;
    for (double x : v_) s += x * x;
    return s;
  }
  double norm() const { return std::sqrt(squaredNorm()); }
  double sum() const {
    double s = 0.0;
    for (double x : v_) s += x;
    return s;
  }
  bool isZero(double tol) const {  // Eigen: max |x_i| <= tol
    for (double x : v_)
      if (std::fabs(x) > tol) return false;
    return true;
  }

  bool operator==(const VectorXd& o) const { return v_ == o.v_; }
  bool operator!=(const VectorXd& o) const { return v_ != o.v_; }
  VectorXd operator+(const VectorXd& o) const {
    VectorXd r(*this);
    return r += o;
  }
  VectorXd operator-(const VectorXd& o) const {
    VectorXd r(*this);
    return r -= o;
  }
  VectorXd& operator+=(const VectorXd& o) {
    for (size_t i = 0; i < v_.size(); ++i) v_[i] += o.v_[i];
    return *this;
  }
  VectorXd& operator-=(const VectorXd& o) {
    for (size_t i = 0; i < v_.size(); ++i) v_[i] -= o.v_[i];
    return *this;
  }
  VectorXd operator*(double s) const {
    VectorXd r(*this);
    for (double& x : r.v_) x *= s;
    return r;
  }
  VectorXd operator-() const { return *this * -1.0; }

 private:
  std::vector<double> v_;
};

inline VectorXd operator*(double s, const VectorXd& v) { return v * s; }

inline std::ostream& operator<<(std::ostream& os, const VectorXd& v) {
  for (Index i = 0; i < v.size(); ++i) os << (i ? "\n" : "") << v[i];
  return os;
}

// Dense column-major matrix of doubles (Eigen::MatrixXd subset).
class MatrixXd {
 public:
  MatrixXd() = default;
  MatrixXd(Index rows, Index cols) : r_(rows), c_(cols), m_((size_t)(rows * cols), 0.0) {}

  static MatrixXd Zero(Index rows, Index cols) { return MatrixXd(rows, cols); }
  static MatrixXd Identity(Index rows, Index cols) {
    MatrixXd m(rows, cols);
    for (Index i = 0; i < rows && i < cols; ++i) m(i, i) = 1.0;
    return m;
  }

  Index rows() const { return r_; }
  Index cols() const { return c_; }
  Index size() const { return r_ * c_; }
  double& operator()(Index i, Index j) { return m_[(size_t)(j * r_ + i)]; }
  double operator()(Index i, Index j) const { return m_[(size_t)(j * r_ + i)]; }
  double* data() { return m_.data(); }
  const double* data() const { return m_.data(); }

  void resize(Index rows, Index cols) {
    r_ = rows;
    c_ = cols;
    m_.assign((size_t)(rows * cols), 0.0);
  }
  MatrixXd& setZero() {
    for (double& x : m_) x = 0.0;
    return *this;
  }
  MatrixXd transpose() const {
    MatrixXd t(c_, r_);
    for (Index i = 0; i < r_; ++i)
      for (Index j = 0; j < c_; ++j) t(j, i) = (*this)(i, j);
    return t;
  }
  MatrixXd operator*(const MatrixXd& o) const {
    MatrixXd p(r_, o.c_);
    for (Index j = 0; j < o.c_; ++j)
      for (Index k = 0; k < c_; ++k) {
        const double b = o(k, j);
        if (b == 0.0) continue;
        for (Index i = 0; i < r_; ++i) p(i, j) += (*this)(i, k) * b;
      }
    return p;
  }
  VectorXd operator*(const VectorXd& v) const {
    VectorXd p(r_);
    for (Index k = 0; k < c_; ++k)
      for (Index i = 0; i < r_; ++i) p[i] += (*this)(i, k) * v[k];
    return p;
  }
  MatrixXd operator-(const MatrixXd& o) const {
    MatrixXd d(*this);
    for (size_t i = 0; i < m_.size(); ++i) d.m_[i] -= o.m_[i];
    return d;
  }
  double maxAbs() const {
    double m = 0.0;
    for (double x : m_) m = std::fabs(x) > m ? std::fabs(x) : m;
    return m;
  }
  bool operator==(const MatrixXd& o) const { return r_ == o.r_ && c_ == o.c_ && m_ == o.m_; }

 private:
  Index r_ = 0, c_ = 0;
  std::vector<double> m_;
};

inline std::ostream& operator<<(std::ostream& os, const MatrixXd& m) {
  for (Index i = 0; i < m.rows(); ++i) {
    for (Index j = 0; j < m.cols(); ++j) os << (j ? " " : "") << m(i, j);
    if (i + 1 < m.rows()) os << "\n";
  }
  return os;
}

// Eigen::Matrix<double, R, C> stand-in (PolynomialOptimization<N>::SquareMatrix).
template <int R, int C>
class FixedMatrix : public MatrixXd {
 public:
  FixedMatrix() : MatrixXd(R, C) {}
  FixedMatrix(const MatrixXd& m) : MatrixXd(m) {}  // NOLINT: Eigen converts implicitly too
};

}  // namespace mav_trajectory_generation
#endif  // MTG_USE_EIGEN

#endif  // MAV_TRAJECTORY_GENERATION_LINALG_H_
