// linalg.h -- the vector / matrix types of the drop-in API.
//
// The reference's public types are Eigen's (Eigen::VectorXd for constraint values and
// coefficients, Eigen::MatrixXd for getA/getM/getR/..., vertex.h:45, polynomial.h:52,
// polynomial_optimization_linear.h:180-214).  When Eigen is on the include path (<Eigen/Core>, or
// <eigen3/Eigen/Core> as the reference includes it, vertex.h:25) the drop-in uses Eigen's own
// types, so a reference caller passes its Eigen::VectorXd / Eigen::MatrixXd unchanged
// (MTG_USE_EIGEN; tests/test_eigen_api.py builds that mode).  Define MTG_NO_EIGEN to opt out, or
// MTG_USE_EIGEN to require Eigen.  Without Eigen (this image has none) the drop-in uses the two
// small dense types below: a strict subset of Eigen's interface (every call the headers make on
// them is valid Eigen too), with zero-initialised storage.
#ifndef MAV_TRAJECTORY_GENERATION_LINALG_H_
#define MAV_TRAJECTORY_GENERATION_LINALG_H_

#if !defined(MTG_USE_EIGEN) && !defined(MTG_NO_EIGEN) && defined(__has_include)
#if __has_include(<Eigen/Core>) || __has_include(<eigen3/Eigen/Core>)
#define MTG_USE_EIGEN 1
#endif
#endif

#ifdef MTG_USE_EIGEN
#if __has_include(<Eigen/Core>)
#include <Eigen/Core>
#else
#include <eigen3/Eigen/Core>
#endif

namespace mav_trajectory_generation {
typedef Eigen::Index Index;
typedef Eigen::VectorXd VectorXd;
typedef Eigen::MatrixXd MatrixXd;
template <int R, int C>
using FixedMatrix = Eigen::Matrix<double, R, C>;
// the allocator of containers of fixed-size matrices (polynomial_optimization_linear.h:53-54)
template <typename T>
using AlignedAllocator = Eigen::aligned_allocator<T>;
}  // namespace mav_trajectory_generation

#else
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <memory>
#include <ostream>
#include <vector>

namespace mav_trajectory_generation {

typedef std::ptrdiff_t Index;
template <typename T>
using AlignedAllocator = std::allocator<T>;  // (Eigen mode: Eigen::aligned_allocator)

namespace detail {
// sum of x_i * y_i in Eigen's reduction order for SSE2 packets of two doubles
// (Eigen/src/Core/Redux.h), so norm() gives the bits Eigen::VectorXd::norm() gives on x86-64
inline double redux_dot(const double* x, const double* y, Index n) {
  if (n <= 0) return 0.0;
  const Index aligned2 = (n / 4) * 4, aligned = (n / 2) * 2;
  if (!aligned) return x[0] * y[0];
  double p0a = x[0] * y[0], p0b = x[1] * y[1];
  if (aligned > 2) {
    double p1a = x[2] * y[2], p1b = x[3] * y[3];
    for (Index i = 4; i < aligned2; i += 4) {
      p0a += x[i] * y[i];
      p0b += x[i + 1] * y[i + 1];
      p1a += x[i + 2] * y[i + 2];
      p1b += x[i + 3] * y[i + 3];
    }
    p0a += p1a;
    p0b += p1b;
    if (aligned > aligned2) {
      p0a += x[aligned2] * y[aligned2];
      p0b += x[aligned2 + 1] * y[aligned2 + 1];
    }
  }
  double res = p0a + p0b;
  for (Index i = aligned; i < n; ++i) res += x[i] * y[i];
  return res;
}

// Eigen's comma initializer: `v << 1, 2, 3;` fills the coefficients in row-major order and the
// count must equal the size (Eigen asserts; here a wrong count aborts).
template <typename M>
class CommaInitializer {
 public:
  CommaInitializer(M& m, double s) : m_(m) { put(s); }
  CommaInitializer(const CommaInitializer&) = delete;
  CommaInitializer& operator,(double s) {
    put(s);
    return *this;
  }
  ~CommaInitializer() {
    if (n_ != m_.size()) std::abort();
  }
  M& finished() { return m_; }

 private:
  void put(double s) {
    if (n_ >= m_.size()) std::abort();
    m_(n_ / m_.cols(), n_ % m_.cols()) = s;
    ++n_;
  }
  M& m_;
  Index n_ = 0;
};
}  // namespace detail

// Dense column vector of doubles (Eigen::VectorXd subset).  New storage is zero-initialised.
class VectorXd {
 public:
  VectorXd() = default;
  explicit VectorXd(Index n) : v_((size_t)n, 0.0) {}

  static VectorXd Zero(Index n) { return VectorXd(n); }
  static VectorXd Ones(Index n) { return Constant(n, 1.0); }
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
  double& operator()(Index i, Index) { return v_[(size_t)i]; }  // (for the comma initializer)
  double* data() { return v_.data(); }
  const double* data() const { return v_.data(); }

  void resize(Index n) { v_.assign((size_t)n, 0.0); }
  VectorXd& setZero() { return setConstant(0.0); }
  VectorXd& setOnes() { return setConstant(1.0); }
  VectorXd& setConstant(double value) {
    for (double& x : v_) x = value;
    return *this;
  }
  // (Eigen returns writable block expressions; these are copies, so only reads compile)
  const VectorXd segment(Index start, Index n) const {
    VectorXd r(n);
    for (Index i = 0; i < n; ++i) r.v_[(size_t)i] = v_[(size_t)(start + i)];
    return r;
  }
  const VectorXd head(Index n) const { return segment(0, n); }
  const VectorXd tail(Index n) const { return segment(size() - n, n); }
  const VectorXd reverse() const {
    VectorXd r(size());
    for (Index i = 0; i < size(); ++i) r.v_[(size_t)i] = v_[(size_t)(size() - 1 - i)];
    return r;
  }
  double dot(const VectorXd& o) const { return detail::redux_dot(data(), o.data(), size()); }
  double squaredNorm() const { return dot(*this); }
  double norm() const { return std::sqrt(squaredNorm()); }
  VectorXd normalized() const {
    const double z = squaredNorm();
    return z > 0.0 ? *this / std::sqrt(z) : *this;
  }
  void normalize() { *this = normalized(); }
  double sum() const {
    double s = 0.0;
    for (double x : v_) s += x;
    return s;
  }
  double maxCoeff() const {
    double m = v_.at(0);
    for (double x : v_) m = x > m ? x : m;
    return m;
  }
  double minCoeff() const {
    double m = v_.at(0);
    for (double x : v_) m = x < m ? x : m;
    return m;
  }
  VectorXd cwiseAbs() const {
    VectorXd r(*this);
    for (double& x : r.v_) x = std::fabs(x);
    return r;
  }
  bool isZero(double tol = 1e-12) const {  // Eigen: max |x_i| <= tol
    for (double x : v_)
      if (std::fabs(x) > tol) return false;
    return true;
  }
  bool isApprox(const VectorXd& o, double prec = 1e-12) const {  // Eigen's definition
    return (*this - o).squaredNorm() <= prec * prec * std::fmin(squaredNorm(), o.squaredNorm());
  }
  bool allFinite() const {
    for (double x : v_)
      if (!std::isfinite(x)) return false;
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
  VectorXd& operator*=(double s) {
    for (double& x : v_) x *= s;
    return *this;
  }
  VectorXd& operator/=(double s) {
    for (double& x : v_) x /= s;
    return *this;
  }
  VectorXd operator*(double s) const {
    VectorXd r(*this);
    return r *= s;
  }
  VectorXd operator/(double s) const {
    VectorXd r(*this);
    return r /= s;
  }
  VectorXd operator-() const { return *this * -1.0; }
  detail::CommaInitializer<VectorXd> operator<<(double s) { return detail::CommaInitializer<VectorXd>(*this, s); }

 private:
  std::vector<double> v_;
};

inline VectorXd operator*(double s, const VectorXd& v) { return v * s; }

inline std::ostream& operator<<(std::ostream& os, const VectorXd& v) {
  for (Index i = 0; i < v.size(); ++i) os << (i ? "\n" : "") << v[i];
  return os;
}

// Dense column-major matrix of doubles (Eigen::MatrixXd subset).  New storage is zero-initialised.
class MatrixXd {
 public:
  MatrixXd() = default;
  MatrixXd(Index rows, Index cols) : r_(rows), c_(cols), m_((size_t)(rows * cols), 0.0) {}

  static MatrixXd Zero(Index rows, Index cols) { return MatrixXd(rows, cols); }
  static MatrixXd Constant(Index rows, Index cols, double value) {
    MatrixXd m(rows, cols);
    for (double& x : m.m_) x = value;
    return m;
  }
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
  MatrixXd& setIdentity() {
    setZero();
    for (Index i = 0; i < r_ && i < c_; ++i) (*this)(i, i) = 1.0;
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
  MatrixXd operator*(double s) const {
    MatrixXd d(*this);
    for (double& x : d.m_) x *= s;
    return d;
  }
  MatrixXd operator+(const MatrixXd& o) const {
    MatrixXd d(*this);
    for (size_t i = 0; i < m_.size(); ++i) d.m_[i] += o.m_[i];
    return d;
  }
  MatrixXd operator-(const MatrixXd& o) const {
    MatrixXd d(*this);
    for (size_t i = 0; i < m_.size(); ++i) d.m_[i] -= o.m_[i];
    return d;
  }
  MatrixXd cwiseAbs() const {
    MatrixXd d(*this);
    for (double& x : d.m_) x = std::fabs(x);
    return d;
  }
  double maxCoeff() const {
    double m = m_.at(0);
    for (double x : m_) m = x > m ? x : m;
    return m;
  }
  bool isZero(double tol = 1e-12) const {
    for (double x : m_)
      if (std::fabs(x) > tol) return false;
    return true;
  }
  bool operator==(const MatrixXd& o) const { return r_ == o.r_ && c_ == o.c_ && m_ == o.m_; }
  bool operator!=(const MatrixXd& o) const { return !(*this == o); }
  detail::CommaInitializer<MatrixXd> operator<<(double s) { return detail::CommaInitializer<MatrixXd>(*this, s); }

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
