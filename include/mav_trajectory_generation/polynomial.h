// polynomial.h -- Polynomial (reference polynomial.h:36-258, src/polynomial.cpp).
//
// Coefficients in increasing powers: c_0 + c_1 t + ... + c_{N-1} t^{N-1}.  evaluate() is the
// reference's Horner on base_coefficients_(d, j) c_j, multiply then add (the library is built with
// -ffp-contract=off, and so must callers that want its last bits).
//
// Not provided: computeRoots / computeMinMax* / selectMinMax* (Jenkins-Traub root finding,
// src/rpoly.cpp, outside the ported path): extrema of whole trajectories go through
// Trajectory::computeMinMaxMagnitude (host or GPU, ExecutionPolicy).
#ifndef MAV_TRAJECTORY_GENERATION_POLYNOMIAL_H_
#define MAV_TRAJECTORY_GENERATION_POLYNOMIAL_H_

#include <algorithm>
#include <cmath>
#include <limits>
#include <vector>

#include "mav_trajectory_generation/linalg.h"
#include "mav_trajectory_generation/runtime.h"

namespace mav_trajectory_generation {

class Polynomial {
 public:
  typedef std::vector<Polynomial> Vector;

  static constexpr int kMaxN = 12;
  static constexpr int kMaxConvolutionSize = 2 * kMaxN - 2;

  // B(n, i) = i! / (i - n)!, 0 for i < n: computeBaseCoefficients (src/polynomial.cpp:140-155),
  // the static base_coefficients_ (kMaxConvolutionSize square, :177-178)
  static double baseCoefficient(int n, int i) {
    if (i < n || n < 0) return 0.0;
    double out = 1.0;
    for (int k = i - n + 1; k <= i; ++k) out *= (double)k;
    return out;
  }
  static MatrixXd computeBaseCoefficients(int n) {
    MatrixXd m = MatrixXd::Zero(n, n);
    for (int r = 0; r < n; ++r)
      for (int i = 0; i < n; ++i) m(r, i) = baseCoefficient(r, i);
    return m;
  }
  static inline MatrixXd base_coefficients_ = computeBaseCoefficients(kMaxConvolutionSize);

  explicit Polynomial(int N) : N_(N), coefficients_(VectorXd::Zero(N)) {}
  Polynomial(int N, const VectorXd& coeffs) : N_(N), coefficients_(coeffs) {
    if ((int)coeffs.size() != N) fail(MTG_ERR_SIZE_MISMATCH, "Number of coefficients has to match.");
  }
  explicit Polynomial(const VectorXd& coeffs) : N_((int)coeffs.size()), coefficients_(coeffs) {}

  int N() const { return N_; }

  bool operator==(const Polynomial& rhs) const { return coefficients_ == rhs.coefficients_; }
  bool operator!=(const Polynomial& rhs) const { return !operator==(rhs); }
  Polynomial operator+(const Polynomial& rhs) const { return Polynomial(VectorXd(coefficients_ + rhs.coefficients_)); }
  Polynomial& operator+=(const Polynomial& rhs) {
    coefficients_ += rhs.coefficients_;
    return *this;
  }
  Polynomial operator*(const Polynomial& rhs) const { return Polynomial(convolve(coefficients_, rhs.coefficients_)); }
  Polynomial operator*(const double& rhs) const { return Polynomial(VectorXd(coefficients_ * rhs)); }

  void setCoefficients(const VectorXd& coeffs) {
    if ((int)coeffs.size() != N_) fail(MTG_ERR_SIZE_MISMATCH, "Number of coefficients has to match.");
    coefficients_ = coeffs;
  }

  // Coefficients of the derivative-th derivative, padded with zeros to N (polynomial.h:100-117).
  VectorXd getCoefficients(int derivative = 0) const {
    if (derivative > N_) fail(MTG_ERR_INVALID_ARGUMENT, "derivative must be <= N");
    if (derivative == 0) return coefficients_;
    VectorXd result = VectorXd::Zero(N_);
    for (int j = 0; j < N_ - derivative; ++j)
      result[j] = coefficients_[j + derivative] * baseCoefficient(derivative, j + derivative);
    return result;
  }

  // Derivatives 0 .. result->size()-1 at t (polynomial.h:120-136).
  void evaluate(double t, VectorXd* result) const {
    check_notnull(result, "result");
    if ((int)result->size() > N_) fail(MTG_ERR_SIZE_MISMATCH, "result size must be <= N");
    const int max_deg = (int)result->size();
    for (int i = 0; i < max_deg; ++i) (*result)[i] = evaluate(t, i);
  }

  // Horner on B(derivative, j) c_j (polynomial.h:138-151).
  double evaluate(double t, int derivative) const {
    if (derivative >= N_) return 0.0;
    const int tmp = N_ - 1;
    if (N_ > kMaxConvolutionSize) {  // beyond the table (the reference would read out of range)
      double result = baseCoefficient(derivative, tmp) * coefficients_[tmp];
      for (int j = tmp - 1; j >= derivative; --j) {
        result *= t;
        result += baseCoefficient(derivative, j) * coefficients_[j];
      }
      return result;
    }
    const MatrixXd& B = base_coefficients_;
    double result = B(derivative, tmp) * coefficients_[tmp];
    for (int j = tmp - 1; j >= derivative; --j) {
      result *= t;
      result += B(derivative, j) * coefficients_[j];
    }
    return result;
  }

  // Row `derivative` of A(t): B(derivative, j) t^(j - derivative); only the j == derivative entry
  // when |t| < epsilon (polynomial.h:215-243).
  static void baseCoeffsWithTime(int N, int derivative, double t, VectorXd* coeffs) {
    check_notnull(coeffs, "coeffs");
    if (derivative < 0 || derivative >= N) fail(MTG_ERR_INVALID_ARGUMENT, "derivative must be in [0, N)");
    coeffs->resize(N);
    coeffs->setZero();
    (*coeffs)[derivative] = baseCoefficient(derivative, derivative);
    if (std::abs(t) < std::numeric_limits<double>::epsilon()) return;
    double t_power = t;
    for (int j = derivative + 1; j < N; j++) {
      (*coeffs)[j] = baseCoefficient(derivative, j) * t_power;
      t_power = t_power * t;
    }
  }
  static VectorXd baseCoeffsWithTime(int N, int derivative, double t) {
    VectorXd c(N);
    baseCoeffsWithTime(N, derivative, t, &c);
    return c;
  }

  // Full discrete convolution (src/polynomial.cpp:157-175).
  static VectorXd convolve(const VectorXd& data, const VectorXd& kernel) {
    const int nd = (int)data.size(), nk = (int)kernel.size();
    VectorXd out = VectorXd::Zero(getConvolutionLength(nd, nk));
    for (int i = 0; i < nd; ++i)
      for (int k = 0; k < nk; ++k) out[i + k] += data[i] * kernel[k];
    return out;
  }
  static int getConvolutionLength(int data_size, int kernel_size) { return data_size + kernel_size - 1; }

 private:
  int N_;
  VectorXd coefficients_;
};

}  // namespace mav_trajectory_generation

#endif  // MAV_TRAJECTORY_GENERATION_POLYNOMIAL_H_
