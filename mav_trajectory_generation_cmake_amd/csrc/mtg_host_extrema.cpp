// mtg_host_extrema.cpp -- host (CPU) path of mtg_min_max_magnitude_batch:
// mtg_host_min_max_magnitude_batch, the reference's Trajectory::computeMinMaxMagnitude
// (src/trajectory.cpp:181-218) for the drop-in's single trajectories, which the reference also
// computes on the CPU.  Same algorithm as the HIP kernel (mtg_extrema.hip): per segment the
// candidates t = 0, t = T and the real roots in [0, T] of sum_d conv(p_d^(k), p_d^(k+1)) (one
// dimension: of p^(k+1)), isolated by sign changes on 256 uniform samples and refined by safeguarded
// Newton-bisection; the magnitude at each candidate; the first candidate / segment wins ties.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <thread>
#include <vector>

#include "mtg.h"
#include "mtg_host_threads.h"

namespace {

constexpr int kSamples = 256;

double ff(int j, int n) {  // falling factorial j! / (j - n)!
  double f = 1.0;
  for (int q = 0; q < n; ++q) f *= (double)(j - q);
  return f;
}

double horner(const double* c, int len, double t) {
  double acc = 0.0;
  for (int j = len - 1; j >= 0; --j) acc = acc * t + c[j];
  return acc;
}

struct Ext {
  double t, v;
};

// one trajectory: coeffs [K][D][N], times [K]
void one(int N, int D, int K, const double* coeffs, const double* times, int k, unsigned dims, mtg_extremum* out_min,
         mtg_extremum* out_max) {
  const int nd = N - k, ndd = N - k - 1;
  const int ndim = __builtin_popcount(dims);
  Ext m{0.0, DBL_MAX}, M{0.0, -DBL_MAX};
  int im = 0, iM = 0;
  std::vector<double> f(2 * N), q(N), q1(N);
  for (int i = 0; i < K; ++i) {
    const double T = times[i];
    const double* cs = coeffs + (size_t)i * D * N;
    for (double& x : f) x = 0.0;
    int lf = 0;
    for (int d = 0; d < D; ++d) {
      if (!((dims >> d) & 1u)) continue;
      for (int j = 0; j < N; ++j) {
        q[j] = j < nd ? cs[d * N + j + k] * ff(j + k, k) : 0.0;
        q1[j] = j < ndd ? cs[d * N + j + k + 1] * ff(j + k + 1, k + 1) : 0.0;
      }
      if (ndim == 1) {  // one dimension: the roots of p^(k+1) (segment.cpp:124-130)
        for (int j = 0; j < ndd; ++j) f[j] = q1[j];
        lf = ndd;
      } else {  // convolve(d, dd) summed over the dimensions
        for (int a = 0; a < nd; ++a)
          for (int c = 0; c < ndd; ++c) f[a + c] += q[a] * q1[c];
        lf = nd + ndd - 1;
      }
    }
    auto mag = [&](double t) {
      double s = 0.0;
      for (int d = 0; d < D; ++d) {
        if (!((dims >> d) & 1u)) continue;
        double acc = 0.0;
        for (int j = nd - 1; j >= 0; --j) acc = acc * t + cs[d * N + j + k] * ff(j + k, k);
        s += acc * acc;
      }
      return std::sqrt(s);
    };
    Ext lo{0.0, DBL_MAX}, hi{0.0, -DBL_MAX};
    auto consider = [&](double t) {
      const double v = mag(t);
      if (v > hi.v) hi = Ext{t, v};
      if (v < lo.v) lo = Ext{t, v};
    };
    consider(0.0);  // t_start, t_end first (polynomial.cpp:38-39), then the roots in order
    consider(T);
    const double h = T / kSamples;
    double ta = 0.0, fa = horner(f.data(), lf, 0.0);
    if (fa == 0.0) consider(0.0);
    for (int s = 1; s <= kSamples; ++s) {
      const double tb = s == kSamples ? T : s * h;
      const double fb = horner(f.data(), lf, tb);
      if (fb == 0.0) {
        consider(tb);
      } else if ((fa < 0.0 && fb > 0.0) || (fa > 0.0 && fb < 0.0)) {
        double a0 = ta, b0 = tb, fa0 = fa, x = ta - fa * ((tb - ta) / (fb - fa));  // from the secant point
        if (!(x > ta && x < tb)) x = 0.5 * (ta + tb);
        for (int it = 0; it < 60; ++it) {
          double fx = 0.0, dfx = 0.0, ga = 0.0;  // f and f' in one Horner pass; ga: f(x)'s error scale
          const double ax = std::fabs(x);
          for (int j = lf - 1; j >= 0; --j) {
            dfx = dfx * x + fx;
            fx = fx * x + f[j];
            ga = ga * ax + std::fabs(f[j]);
          }
          if (std::fabs(fx) <= (2.0 * (2 * N - 2) * DBL_EPSILON) * ga) break;  // within rounding of 0
          if ((fx < 0.0) == (fa0 < 0.0)) a0 = x, fa0 = fx;
          else b0 = x;
          double xn = x - fx / dfx;
          if (!(xn > a0 && xn < b0)) xn = 0.5 * (a0 + b0);
          if (b0 - a0 <= 4.0 * DBL_EPSILON * std::fmax(std::fabs(a0), std::fabs(b0)) || xn == x) {
            x = xn;
            break;
          }
          x = xn;
        }
        consider(x);
      }
      ta = tb;
      fa = fb;
    }
    if (i == 0 || lo.v < m.v) m = lo, im = i;  // strict: the first segment wins ties
    if (i == 0 || hi.v > M.v) M = hi, iM = i;
  }
  if (out_min) *out_min = mtg_extremum{m.t, m.v, im, 0};
  if (out_max) *out_max = mtg_extremum{M.t, M.v, iM, 0};
}

}  // namespace

extern "C" int mtg_host_min_max_magnitude_batch(int N, int D, int K, int64_t batch, const double* coeffs,
                                                const double* times, int derivative, uint32_t dimension_mask,
                                                mtg_extremum* minimum, mtg_extremum* maximum, int threads) {
  if (N < 2 || N > 12 || (N % 2)) return MTG_ERR_UNSUPPORTED_N;
  if (K < 1 || D < 1 || batch < 0) return MTG_ERR_SIZE_MISMATCH;
  if (derivative < 0 || derivative > N - 2) return MTG_ERR_BAD_DERIVATIVE;
  const uint32_t all = D >= 32 ? 0xffffffffu : ((1u << D) - 1u);
  const uint32_t dims = dimension_mask ? dimension_mask : all;
  if (D > 32 || (dims & ~all)) return MTG_ERR_INVALID_ARGUMENT;
  if (batch == 0) return MTG_OK;
  if (!coeffs || !times) return MTG_ERR_INVALID_ARGUMENT;
  const size_t sc = (size_t)K * D * N;
  auto run = [&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b)
      one(N, D, K, coeffs + b * sc, times + b * K, derivative, dims, minimum ? minimum + b : nullptr,
          maximum ? maximum + b : nullptr);
  };
  int nt = threads > 0 ? threads : mtg::usable_cpus();
  if (nt < 1) nt = 1;
  if ((int64_t)nt > batch) nt = (int)batch;
  if (nt == 1) {
    run(0, batch);
    return MTG_OK;
  }
  std::vector<std::thread> pool;
  const int64_t per = (batch + nt - 1) / nt;
  for (int t = 1; t < nt; ++t) {
    const int64_t b0 = std::min<int64_t>(batch, t * per), b1 = std::min<int64_t>(batch, b0 + per);
    try {
      pool.emplace_back(run, b0, b1);
    } catch (...) {
      run(b0, b1);
    }
  }
  run(0, std::min<int64_t>(batch, per));
  for (auto& th : pool) th.join();
  return MTG_OK;
}
