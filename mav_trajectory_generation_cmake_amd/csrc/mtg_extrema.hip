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
// Here: a group of L lanes per (trajectory, segment) (L = 16 lanes of one wave for K <= 32; the
// block holds whole trajectories).  The real roots in [0, T] are isolated by the sign changes of the
// root polynomial f on kExtremaSamples + 1 uniform samples -- lane l of the group evaluates f on its
// own run of kExtremaSamples / L sample intervals -- and refined by safeguarded Newton-bisection to a
// few ulp.  The reference's own test checks its candidates the same way, against sampled extrema
// (test/test_polynomial_optimization.cpp:447-487).  A root pair closer than T / kExtremaSamples (no
// sign change between samples) is not isolated; at such a pair |p^(k)| is flat to second order, so
// the extreme values move by O((T/S)^2) relative.
//
// Work layout (the SIMT costs dominated a direct version by ~10x):
// * f = sum_d conv(p_d^(k), p_d^(k+1)) is formed once per group, each lane its share of the
//   coefficients (f[n], n = lane mod L), from the derivative coefficients staged in LDS dimension by
//   dimension -- not by every lane of the group;
// * a lane first scans its samples and only records the sign-change brackets (up to kMaxBrackets;
//   more are refined in the scan); then all lanes refine their brackets at the same time, so a wave
//   runs the Newton loop once per bracket a lane holds (~1) instead of once per distinct sample index
//   with a root anywhere in the wave (~8 at config 2);
// * the derivative coefficient factors j!/(j-k)! come from a table.
// Candidates carry their position in the sequential order (t = 0, t = T, then the roots by sample
// index), and the group's minimum and maximum are reduced across lanes with that order as the
// tie-break: the same candidate wins as in a sequential scan (std::max / std::min keep the earlier
// candidate on ties).
#include "mtg_device.h"

namespace mtg {

constexpr int kExtremaSamples = 256;
constexpr int kExtremaMaxThreads = 512;
constexpr int kMaxBrackets = 4;

// falling factorials j!/(j-k)!, j, k < 12 (exact in FP64)
struct FallingTable {
  double v[12][12];
};
constexpr FallingTable make_falling_table() {
  FallingTable t{};
  for (int j = 0; j < 12; ++j)
    for (int k = 0; k < 12; ++k) {
      double f = 1.0;
      for (int q = 0; q < k; ++q) f *= (double)(j - q);
      t.v[j][k] = k > j ? 0.0 : f;
    }
  return t;
}
static __constant__ FallingTable c_ff = make_falling_table();

namespace {

struct Ext {
  double t, v;
  int ord;  // position in the sequential candidate order (tie-break)
};

// Horner over the whole zero-padded array: leading zero coefficients leave acc exactly 0, so the
// value is the same as over the first len terms, without a select per term
template <int L>
__device__ __forceinline__ double horner(const double (&c)[L], double t) {
  double acc = 0.0;
#pragma unroll
  for (int j = L - 1; j >= 0; --j) acc = acc * t + c[j];
  return acc;
}

// a beats b as the maximum (larger value; on a tie the earlier candidate)
__device__ __forceinline__ bool better_max(const Ext& a, const Ext& b) { return a.v > b.v || (a.v == b.v && a.ord < b.ord); }
__device__ __forceinline__ bool better_min(const Ext& a, const Ext& b) { return a.v < b.v || (a.v == b.v && a.ord < b.ord); }

__device__ __forceinline__ Ext shfl_xor(const Ext& e, int m, int width) {
  return Ext{__shfl_xor(e.t, m, width), __shfl_xor(e.v, m, width), __shfl_xor(e.ord, m, width)};
}

// safeguarded Newton-bisection on [ta, tb] (a sign change of f, f(ta) = fa), to a few ulp
template <int LF>
__device__ __forceinline__ double refine(const double (&f)[LF], const double (&fp)[LF], double ta, double tb,
                                         double fa) {
  double a0 = ta, b0 = tb, fa0 = fa, x = 0.5 * (ta + tb);
  for (int it = 0; it < 60; ++it) {
    const double fx = horner<LF>(f, x);
    if (fx == 0.0) break;
    if ((fx < 0.0) == (fa0 < 0.0)) a0 = x, fa0 = fx;
    else b0 = x;
    const double dfx = horner<LF>(fp, x);
    double xn = x - fx / dfx;
    if (!(xn > a0 && xn < b0)) xn = 0.5 * (a0 + b0);
    if (b0 - a0 <= 4.0 * DBL_EPSILON * fmax(fabs(a0), fabs(b0)) || xn == x) {
      x = xn;
      break;
    }
    x = xn;
  }
  return x;
}

// L lanes per (trajectory, segment); tpb whole trajectories per block.  LDS per group: the root
// polynomial f [LF] and one dimension's derivative coefficients q, q1 [2 N]; then the groups' extremes.
template <int N, int L>
__global__ __launch_bounds__(kExtremaMaxThreads) void min_max_magnitude_kernel(
    const double* __restrict__ coeffs, const double* __restrict__ times, int64_t B, int K, int D, int k,
    unsigned dims, int tpb, mtg_extremum* __restrict__ out_min, mtg_extremum* __restrict__ out_max) {
  constexpr int LF = 2 * N - 2;             // root polynomial length bound (conv of N and N-1 terms)
  constexpr int SPL = kExtremaSamples / L;  // sample intervals per lane
  constexpr int GS = LF + 2 * N;            // LDS doubles per group
  constexpr int UF = (LF + L - 1) / L;      // f coefficients per lane
  extern __shared__ __attribute__((aligned(16))) double xlds[];
  const int tid = threadIdx.x;
  const int lane = tid % L, grp = tid / L;  // the group of L lanes owns one (trajectory, segment)
  const int ngrp = tpb * K;                 // groups of the block
  const int bl = grp / K, i = grp - bl * K;
  const int64_t b = (int64_t)blockIdx.x * tpb + bl;
  const bool active = grp < ngrp && b < B;
  const int nd = N - k, ndd = N - k - 1;  // p^(k), p^(k+1) coefficient counts
  const int ndim = __builtin_popcount(dims);
  Ext* smin = reinterpret_cast<Ext*>(xlds + (size_t)ngrp * GS);
  Ext* smax = smin + ngrp;
  const int g = grp < ngrp ? grp : 0;
  double* gf = xlds + (size_t)g * GS;  // this group's f, then q, q1
  double* gq = gf + LF;
  double* gq1 = gq + N;

  Ext lo{0.0, DBL_MAX, 0x7fffffff}, hi{0.0, -DBL_MAX, 0x7fffffff};
  const int64_t bb = active ? b : 0;
  const int ii = active ? i : 0;
  const double T = times[bb * K + ii];
  const double* cs = coeffs + ((bb * K + ii) * D) * N;
  // ---- f: lane l forms f[n], n = l, l + L, ..., from q_d, q1_d staged per selected dimension
  double facc[UF];
#pragma unroll
  for (int u = 0; u < UF; ++u) facc[u] = 0.0;
  for (int d = 0; d < D; ++d) {
    if (!((dims >> d) & 1u)) continue;
    for (int j = lane; j < 2 * N; j += L) {
      const int jj = j < N ? j : j - N;
      double v = 0.0;
      if (j < N) {
        if (jj < nd) v = cs[d * N + jj + k] * c_ff.v[jj + k][k];
      } else if (jj < ndd) {
        v = cs[d * N + jj + k + 1] * c_ff.v[jj + k + 1][k + 1];
      }
      if (grp < ngrp) gq[j] = v;
    }
    lds_fence();  // (the group is L consecutive lanes of one wave)
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      const int n = lane + u * L;
      if (n >= LF) continue;
      if (ndim == 1) {  // one dimension: the roots of p^(k+1) (segment.cpp:124-130)
        facc[u] = n < N ? gq1[n] : 0.0;
      } else {  // convolve(d, dd) (polynomial.h convolve), summed over dimensions
        double t = 0.0;
        const int a0 = n - (N - 1) > 0 ? n - (N - 1) : 0, a1 = n < N - 1 ? n : N - 1;
        for (int a = a0; a <= a1; ++a) t += gq[a] * gq1[n - a];
        facc[u] += t;
      }
    }
    lds_fence();  // (read before the next dimension overwrites q, q1)
  }
#pragma unroll
  for (int u = 0; u < UF; ++u) {
    const int n = lane + u * L;
    if (n < LF && grp < ngrp) gf[n] = facc[u];
  }
  lds_fence();
  double f[LF], fp[LF];  // f and f'
#pragma unroll
  for (int j = 0; j < LF; ++j) f[j] = gf[j];
#pragma unroll
  for (int j = 0; j < LF; ++j) fp[j] = (j + 1 < LF) ? f[j + 1] * (double)(j + 1) : 0.0;

  if (active) {
    auto mag = [&](double t) {
      double s = 0.0;
      for (int d = 0; d < D; ++d) {
        if (!((dims >> d) & 1u)) continue;
        double acc = 0.0;
        for (int j = nd - 1; j >= 0; --j) acc = acc * t + cs[d * N + j + k] * c_ff.v[j + k][k];
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
    const double h = T / kExtremaSamples;
    const int s0 = lane * SPL;
    double ta = s0 * h, fa = horner<LF>(f, ta);
    if (s0 == 0 && fa == 0.0) consider(0.0, 2);
    // scan: record the brackets (an overflow is refined in the scan)
    double bta[kMaxBrackets], btb[kMaxBrackets], bfa[kMaxBrackets];
    int bs[kMaxBrackets];
#pragma unroll
    for (int q = 0; q < kMaxBrackets; ++q) bta[q] = btb[q] = bfa[q] = 0.0, bs[q] = 0;
    int nb = 0;
    for (int s = s0 + 1; s <= s0 + SPL; ++s) {
      const double tb = s == kExtremaSamples ? T : s * h;
      const double fb = horner<LF>(f, tb);
      if (fb == 0.0) {
        consider(tb, 2 + s);
      } else if ((fa < 0.0 && fb > 0.0) || (fa > 0.0 && fb < 0.0)) {
        if (nb < kMaxBrackets) {
#pragma unroll
          for (int q = 0; q < kMaxBrackets; ++q)
            if (q == nb) bta[q] = ta, btb[q] = tb, bfa[q] = fa, bs[q] = s;
          ++nb;
        } else {
          consider(refine<LF>(f, fp, ta, tb, fa), 2 + s);
        }
      }
      ta = tb;
      fa = fb;
    }
    // refine: all lanes at once
#pragma unroll
    for (int q = 0; q < kMaxBrackets; ++q)
      if (q < nb) consider(refine<LF>(f, fp, bta[q], btb[q], bfa[q]), 2 + bs[q]);
  }
  // the group's extremes (lanes of one group are consecutive lanes of one wave)
#pragma unroll
  for (int m = L / 2; m >= 1; m >>= 1) {
    const Ext a = shfl_xor(lo, m, L), c = shfl_xor(hi, m, L);
    if (better_min(a, lo)) lo = a;
    if (better_max(c, hi)) hi = c;
  }
  if (lane == 0 && grp < ngrp) smin[grp] = lo, smax[grp] = hi;
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

// lanes per segment and trajectories per block: 16 lanes while a trajectory fits a block (K <= 32),
// then fewer; the trajectories per block that keep the block's waves fullest (K = 10: 16 lanes, 2
// trajectories, 320 threads = 5 full waves)
void extrema_geometry(int K, int* lanes, int* tpb, int* threads) {
  int L = 16;
  while (L > 1 && K * L > kExtremaMaxThreads) L >>= 1;
  int best_t = 1;
  double best_u = 0.0;
  for (int t = 1; t * K * L <= kExtremaMaxThreads; ++t) {
    const int th = (t * K * L + 63) / 64 * 64;
    const double u = (double)(t * K * L) / th;
    if (u > best_u + 1e-9) best_u = u, best_t = t;
  }
  *lanes = L;
  *tpb = best_t;
  *threads = (best_t * K * L + 63) / 64 * 64;
}

template <int N, int L>
hipError_t launch_extrema_nl(const double* coeffs, const double* times, int64_t B, int K, int D, int k, unsigned dims,
                             int tpb, int threads, mtg_extremum* mn, mtg_extremum* mx, hipStream_t stream) {
  const size_t lds = sizeof(double) * (size_t)tpb * K * (2 * N - 2 + 2 * N) + 2 * sizeof(Ext) * (size_t)tpb * K;
  const dim3 grid((unsigned)((B + tpb - 1) / tpb)), block(threads);
  launch_kernel((min_max_magnitude_kernel<N, L>), grid, block, (uint32_t)lds, stream, coeffs, times, B, K, D, k, dims,
                tpb, mn, mx);
  return hipGetLastError();
}

template <int N>
hipError_t launch_extrema_n(const double* coeffs, const double* times, int64_t B, int K, int D, int k, unsigned dims,
                            mtg_extremum* mn, mtg_extremum* mx, hipStream_t stream) {
  int L, tpb, threads;
  extrema_geometry(K, &L, &tpb, &threads);
  switch (L) {
    case 16: return launch_extrema_nl<N, 16>(coeffs, times, B, K, D, k, dims, tpb, threads, mn, mx, stream);
    case 8: return launch_extrema_nl<N, 8>(coeffs, times, B, K, D, k, dims, tpb, threads, mn, mx, stream);
    case 4: return launch_extrema_nl<N, 4>(coeffs, times, B, K, D, k, dims, tpb, threads, mn, mx, stream);
    case 2: return launch_extrema_nl<N, 2>(coeffs, times, B, K, D, k, dims, tpb, threads, mn, mx, stream);
    default: return launch_extrema_nl<N, 1>(coeffs, times, B, K, D, k, dims, tpb, threads, mn, mx, stream);
  }
}

}  // namespace

hipError_t launch_min_max_magnitude(int N, const double* coeffs, const double* times, int64_t B, int K, int D,
                                    int derivative, unsigned dims, mtg_extremum* mn, mtg_extremum* mx,
                                    hipStream_t stream) {
  if (K < 1 || K > 256) return hipErrorInvalidValue;
  if (B == 0) return hipSuccess;
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
