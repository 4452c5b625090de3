// mtg_extrema.hip -- minimum and maximum magnitude of a derivative over whole trajectories
// (mtg_min_max_magnitude_batch): the reference's Trajectory::computeMinMaxMagnitude
// (src/trajectory.cpp:181-218) over Segment::computeMinMaxMagnitudeCandidates /
// selectMinMaxMagnitudeFromCandidates (src/segment.cpp:82-196).
//
// Reference: per segment the candidate times are t = 0, t = T and the real roots in [0, T] of
//   sum_{d in dims} conv(p_d^(k), p_d^(k+1))      (the derivative of |p^(k)|^2 / 2; one selected
//                                                   dimension: the roots of p^(k+1) alone)
// found by Jenkins-Traub (src/rpoly.cpp) with |imag| <= DBL_EPSILON as "real"; the magnitude
// sqrt(sum p_d^(k)(t)^2) is evaluated at every candidate and the segment minimum / maximum taken,
// then the trajectory's (strict comparisons: the first segment wins ties).
//
// Here: a group of L lanes per (trajectory, segment) (L = 8 or 16 lanes of one wave, chosen per K so
// a 256-thread block holds whole trajectories).  The real roots in [0, T] are isolated by the sign
// changes of the root polynomial f on kExtremaSamples + 1 uniform samples -- lane l of the group
// evaluates f on its own run of kExtremaSamples / L sample intervals -- and each bracket is refined
// by safeguarded Newton-bisection to a few ulp on the lane that found it.  The reference's own test
// checks its candidates the same way, against sampled extrema
// (test/test_polynomial_optimization.cpp:447-487).  A root pair closer than T / kExtremaSamples (no
// sign change between samples) is not isolated; at such a pair |p^(k)| is flat to second order, so
// the extreme values move by O((T/S)^2) relative.  Candidates carry their position in the
// sequential order (t = 0, t = T, then the roots by sample index), and the group's minimum and
// maximum are reduced across lanes with that order as the tie-break: the same candidate wins as in
// a sequential scan (std::max / std::min keep the earlier candidate on ties).
#include "mtg_device.h"

namespace mtg {

constexpr int kExtremaSamples = 256;
constexpr int kExtremaThreads = 256;

namespace {

struct Ext {
  double t, v;
  int ord;  // position in the sequential candidate order (tie-break)
};

// falling factorial j!/(j-n)!
__device__ __forceinline__ double ff(int j, int n) {
  double f = 1.0;
  for (int q = 0; q < n; ++q) f *= (double)(j - q);
  return f;
}

template <int L>
__device__ __forceinline__ double horner(const double (&c)[L], int len, double t) {
  double acc = 0.0;
#pragma unroll
  for (int j = L - 1; j >= 0; --j)
    if (j < len) acc = acc * t + c[j];
  return acc;
}

// a beats b as the maximum (larger value; on a tie the earlier candidate)
__device__ __forceinline__ bool better_max(const Ext& a, const Ext& b) { return a.v > b.v || (a.v == b.v && a.ord < b.ord); }
__device__ __forceinline__ bool better_min(const Ext& a, const Ext& b) { return a.v < b.v || (a.v == b.v && a.ord < b.ord); }

__device__ __forceinline__ Ext shfl_xor(const Ext& e, int m, int width) {
  return Ext{__shfl_xor(e.t, m, width), __shfl_xor(e.v, m, width), __shfl_xor(e.ord, m, width)};
}

// L lanes per segment; block = kExtremaThreads threads = TPB whole trajectories of K segments
template <int N, int L>
__global__ __launch_bounds__(kExtremaThreads) void min_max_magnitude_kernel(
    const double* __restrict__ coeffs, const double* __restrict__ times, int64_t B, int K, int D, int k,
    unsigned dims, mtg_extremum* __restrict__ out_min, mtg_extremum* __restrict__ out_max) {
  constexpr int LQ = N;          // derivative polynomial length bound
  constexpr int LF = 2 * N - 2;  // root polynomial length bound (conv of N and N-1 terms)
  constexpr int SPL = kExtremaSamples / L;  // sample intervals per lane
  __shared__ Ext smin[kExtremaThreads / L], smax[kExtremaThreads / L];
  const int tid = threadIdx.x;
  const int lane = tid % L, grp = tid / L;  // the group of L lanes owns one (trajectory, segment)
  const int tpb = (kExtremaThreads / L) / K;  // trajectories per block
  const int bl = grp / K, i = grp - bl * K;
  const int64_t b = (int64_t)blockIdx.x * tpb + bl;
  const bool active = bl < tpb && b < B;
  const int nd = N - k, ndd = N - k - 1;  // p^(k), p^(k+1) coefficient counts
  const int ndim = __builtin_popcount(dims);

  Ext lo{0.0, DBL_MAX, 0x7fffffff}, hi{0.0, -DBL_MAX, 0x7fffffff};
  if (active) {
    const double T = times[b * K + i];
    const double* cs = coeffs + ((b * K + i) * D) * N;
    // root polynomial f, dimension by dimension (every lane of the group forms it)
    double f[LF];
#pragma unroll
    for (int j = 0; j < LF; ++j) f[j] = 0.0;
    int lf = 0;
    for (int d = 0; d < D; ++d) {
      if (!((dims >> d) & 1u)) continue;
      double q[LQ], q1[LQ];
#pragma unroll
      for (int j = 0; j < LQ; ++j) {
        q[j] = j < nd ? cs[d * N + j + k] * ff(j + k, k) : 0.0;
        q1[j] = j < ndd ? cs[d * N + j + k + 1] * ff(j + k + 1, k + 1) : 0.0;
      }
      if (ndim == 1) {  // one dimension: the roots of p^(k+1) (segment.cpp:124-130)
#pragma unroll
        for (int j = 0; j < LF; ++j) f[j] = j < LQ ? q1[j] : 0.0;
        lf = ndd;
      } else {  // convolve(d, dd) (polynomial.h convolve), summed over dimensions
#pragma unroll
        for (int a = 0; a < LQ; ++a)
#pragma unroll
          for (int c = 0; c < LQ; ++c)
            if (a < nd && c < ndd && a + c < LF) f[a + c] += q[a] * q1[c];
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
      return sqrt(s);
    };
    auto consider = [&](double t, int ord) {
      const Ext e{t, mag(t), ord};
      if (better_max(e, hi)) hi = e;
      if (better_min(e, lo)) lo = e;
    };
    // candidates t_start, t_end first (polynomial.cpp:38-39), then the roots in sample order
    if (lane == 0) consider(0.0, 0);
    if (lane == L - 1) consider(T, 1);
    double fp[LF];  // f'
#pragma unroll
    for (int j = 0; j < LF; ++j) fp[j] = (j + 1 < LF) ? f[j + 1] * (double)(j + 1) : 0.0;
    const double h = T / kExtremaSamples;
    const int s0 = lane * SPL;
    double ta = s0 * h, fa = horner<LF>(f, lf, ta);
    if (s0 == 0 && fa == 0.0) consider(0.0, 2);
    for (int s = s0 + 1; s <= s0 + SPL; ++s) {
      const double tb = s == kExtremaSamples ? T : s * h;
      const double fb = horner<LF>(f, lf, tb);
      if (fb == 0.0) {
        consider(tb, 2 + s);
      } else if ((fa < 0.0 && fb > 0.0) || (fa > 0.0 && fb < 0.0)) {
        // safeguarded Newton-bisection on [ta, tb] with f(ta) f(tb) < 0
        double a0 = ta, b0 = tb, fa0 = fa, x = 0.5 * (ta + tb);
        for (int it = 0; it < 60; ++it) {
          const double fx = horner<LF>(f, lf, x);
          if (fx == 0.0) break;
          if ((fx < 0.0) == (fa0 < 0.0)) a0 = x, fa0 = fx;
          else b0 = x;
          const double dfx = horner<LF>(fp, lf - 1, x);
          double xn = x - fx / dfx;
          if (!(xn > a0 && xn < b0)) xn = 0.5 * (a0 + b0);
          if (b0 - a0 <= 4.0 * DBL_EPSILON * fmax(fabs(a0), fabs(b0)) || xn == x) {
            x = xn;
            break;
          }
          x = xn;
        }
        consider(x, 2 + s);
      }
      ta = tb;
      fa = fb;
    }
  }
  // the group's extremes (lanes of one group are consecutive lanes of one wave)
#pragma unroll
  for (int m = L / 2; m >= 1; m >>= 1) {
    const Ext a = shfl_xor(lo, m, L), c = shfl_xor(hi, m, L);
    if (better_min(a, lo)) lo = a;
    if (better_max(c, hi)) hi = c;
  }
  if (lane == 0) smin[grp] = lo, smax[grp] = hi;
  __syncthreads();
  if (active && i == 0 && lane == 0) {  // trajectory's segments in order; strict: the first segment wins ties
    Ext m = smin[grp], M = smax[grp];
    int im = 0, iM = 0;
    for (int q = 1; q < K; ++q) {
      const Ext a = smin[grp + q], c = smax[grp + q];
      if (a.v < m.v) m = a, im = q;
      if (c.v > M.v) M = c, iM = q;
    }
    if (out_min) out_min[b] = mtg_extremum{m.t, m.v, im, 0};
    if (out_max) out_max[b] = mtg_extremum{M.t, M.v, iM, 0};
  }
}

// lanes per segment: the larger of 16 / 8 / 4 / 2 / 1 that keeps a 256-thread block >= 7/8 busy with
// whole trajectories (K = 10: 8 lanes, 3 trajectories per block)
int extrema_lanes(int K) {
  int best = 1;
  double best_util = 0.0;
  for (int L = 16; L >= 1; L >>= 1) {
    if (K * L > kExtremaThreads) continue;
    const int tpb = kExtremaThreads / (K * L);
    const double util = (double)(tpb * K * L) / kExtremaThreads;
    if (util >= 0.875) return L;
    if (util > best_util) best_util = util, best = L;
  }
  return best;
}

template <int N, int L>
hipError_t launch_extrema_nl(const double* coeffs, const double* times, int64_t B, int K, int D, int k, unsigned dims,
                             mtg_extremum* mn, mtg_extremum* mx, hipStream_t stream) {
  const int tpb = (kExtremaThreads / L) / K;
  const dim3 grid((unsigned)((B + tpb - 1) / tpb)), block(kExtremaThreads);
  launch_kernel((min_max_magnitude_kernel<N, L>), grid, block, 0, stream, coeffs, times, B, K, D, k, dims, mn, mx);
  return hipGetLastError();
}

template <int N>
hipError_t launch_extrema_n(const double* coeffs, const double* times, int64_t B, int K, int D, int k, unsigned dims,
                            mtg_extremum* mn, mtg_extremum* mx, hipStream_t stream) {
  switch (extrema_lanes(K)) {
    case 16: return launch_extrema_nl<N, 16>(coeffs, times, B, K, D, k, dims, mn, mx, stream);
    case 8: return launch_extrema_nl<N, 8>(coeffs, times, B, K, D, k, dims, mn, mx, stream);
    case 4: return launch_extrema_nl<N, 4>(coeffs, times, B, K, D, k, dims, mn, mx, stream);
    case 2: return launch_extrema_nl<N, 2>(coeffs, times, B, K, D, k, dims, mn, mx, stream);
    default: return launch_extrema_nl<N, 1>(coeffs, times, B, K, D, k, dims, mn, mx, stream);
  }
}

}  // namespace

hipError_t launch_min_max_magnitude(int N, const double* coeffs, const double* times, int64_t B, int K, int D,
                                    int derivative, unsigned dims, mtg_extremum* mn, mtg_extremum* mx,
                                    hipStream_t stream) {
  if (K < 1 || K > kExtremaThreads || B == 0) return K < 1 || K > kExtremaThreads ? hipErrorInvalidValue : hipSuccess;
  switch (N) {
    case 2: return launch_extrema_n<2>(coeffs, times, B, K, D, derivative, dims, mn, mx, stream);
    case 4: return launch_extrema_n<4>(coeffs, times, B, K, D, derivative, dims, mn, mx, stream);
    case 6: return launch_extrema_n<6>(coeffs, times, B, K, D, derivative, dims, mn, mx, stream);
    case 8: return launch_extrema_n<8>(coeffs, times, B, K, D, derivative, dims, mn, mx, stream);
    case 10: return launch_extrema_n<10>(coeffs, times, B, K, D, derivative, dims, mn, mx, stream);
    case 12: return launch_extrema_n<12>(coeffs, times, B, K, D, derivative, dims, mn, mx, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
