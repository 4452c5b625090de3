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
// Here: a group of L lanes per (trajectory, segment) (L = 8 lanes of one wave for K <= 64; the
// block holds whole trajectories).  The real roots in [0, T] are isolated by the sign changes of the
// root polynomial f on kExtremaSamples + 1 uniform samples -- lane l of the group evaluates f on its
// own run of kExtremaSamples / L sample intervals -- and refined by safeguarded Newton-bisection until
// f is within its rounding error of 0.  The reference's own test checks its candidates the same way, against sampled extrema
// (test/test_polynomial_optimization.cpp:447-487).  A root pair closer than T / kExtremaSamples (no
// sign change between samples) is not isolated; at such a pair |p^(k)| is flat to second order, so
// the extreme values move by O((T/S)^2) relative.
//
// Work layout (latency, not arithmetic, set the cost of the direct versions):
// * the group stages the derivative coefficients q_d = p_d^(k), q1_d = p_d^(k+1) of up to QD selected
//   dimensions in LDS with one batch of loads (QD = 4 unless the block's LDS would not fit), forms
//   f = sum_d conv(q_d, q1_d) there, each lane its share of the coefficients, and evaluates the
//   magnitude at the candidates from the staged q_d (more than QD dimensions: from global memory);
// * the scan only sets bits -- sample intervals with a sign change, samples where f is exactly 0,
//   the end points -- and one loop then takes each lane's candidates lowest bit first, refining the
//   brackets: a wave runs the refinement once per candidate a lane holds (~1), and the Newton
//   iteration, the magnitude and the candidate comparison exist once in the code;
// * the Newton step takes f and f' from one Horner pass.
// Candidates carry their position in the sequential order (t = 0, t = T, then the roots by sample
// index), and the group's minimum and maximum are reduced across lanes with that order as the
// tie-break: the same candidate wins as in a sequential scan (std::max / std::min keep the earlier
// candidate on ties).
#include "mtg_device.h"

namespace mtg {

constexpr int kExtremaSamples = 256;
constexpr int kExtremaMaxThreads = 512;
constexpr int kExtremaQD = 4;  // dimensions staged per pass (at most)
#ifndef MTG_EXTREMA_CS
#define MTG_EXTREMA_CS 16
#endif

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

// LDS doubles of one group: f, then q_d of qd dimensions, then their q1_d with zero pads
__host__ __device__ constexpr int extrema_group_doubles(int N, int qd) { return 2 * N + qd * N + (2 * qd + 1) * N; }

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

// safeguarded Newton-bisection on [ta, tb] (a sign change of f, f(ta) = fa, f(tb) = fb) from the
// secant point, until f(x) is within its rounding error of 0; f and f' from one Horner pass (as
// mtg_host_extrema.cpp)
template <int LF>
__device__ __forceinline__ double refine(const double (&f)[LF], double ta, double tb, double fa, double fb) {
  double a0 = ta, b0 = tb, fa0 = fa, x = ta - fa * ((tb - ta) / (fb - fa));
  if (!(x > ta && x < tb)) x = 0.5 * (ta + tb);
  for (int it = 0; it < 60; ++it) {
    double fx = 0.0, dfx = 0.0, ga = 0.0;  // ga: sum |f_j| |x|^j, the scale of f(x)'s rounding error
    const double ax = fabs(x);
#pragma unroll
    for (int j = LF - 1; j >= 0; --j) {
      dfx = dfx * x + fx;
      fx = fx * x + f[j];
      ga = ga * ax + fabs(f[j]);
    }
    // f(x) indistinguishable from 0 (below its own evaluation error): converged.  Without this the
    // Newton steps wander by the rounding noise and only the bisection bound ends them (~45 steps).
    if (fabs(fx) <= (2.0 * LF * DBL_EPSILON) * ga) break;
    if ((fx < 0.0) == (fa0 < 0.0)) a0 = x, fa0 = fx;
    else b0 = x;
    double xn = x - fx * __builtin_amdgcn_rcp(dfx);  // (a Newton step: an approximate reciprocal will do)
    if (!(xn > a0 && xn < b0)) xn = 0.5 * (a0 + b0);
    if (b0 - a0 <= 4.0 * DBL_EPSILON * fmax(fabs(a0), fabs(b0)) || xn == x) {
      x = xn;
      break;
    }
    x = xn;
  }
  return x;
}

// index of the m-th selected dimension (m-th set bit of dims)
__device__ __forceinline__ int sel_dim(unsigned dims, int m) {
  for (int r = 0; r < m; ++r) dims &= dims - 1u;
  return __builtin_ctz(dims);
}

// L lanes per (trajectory, segment); tpb whole trajectories per block; qd dimensions staged per
// pass.  LDS per group (extrema_group_doubles): f [2N]; q [qd][N]; q1 with zero pads,
// [Z q1_0 Z q1_1 ... q1_{qd-1} Z] (N doubles each), so that the convolution reads q1[n - a] at a
// fixed offset from n for every a, without bounds selects; then the groups' extremes.
// Waves per SIMD the register budget is built for: at N <= 10 five (96 VGPRs, ~14 spilled: config 2,
// L = 8, 0.104 -> 0.089 ms against four without spills); N = 12 spills ~40 at five, so the compiler's
// own choice.
template <int N>
constexpr int extrema_waves() { return N <= 10 ? 5 : 1; }

template <int N, int L>
__global__ __launch_bounds__(kExtremaMaxThreads) __attribute__((amdgpu_waves_per_eu(extrema_waves<N>()))) void min_max_magnitude_kernel(
    const double* __restrict__ coeffs, const double* __restrict__ times, int64_t B, int K, int D, int k,
    unsigned dims, int tpb, int qd, mtg_extremum* __restrict__ out_min, mtg_extremum* __restrict__ out_max) {
  constexpr int LF = 2 * N - 2;             // root polynomial length bound (conv of N and N-1 terms)
  constexpr int SPL = kExtremaSamples / L;  // sample intervals per lane
  constexpr int CH = SPL < 64 ? SPL : 64;   // sample intervals per candidate mask (one bit each)
  constexpr int CS = CH < MTG_EXTREMA_CS ? CH : MTG_EXTREMA_CS;  // sample intervals per unrolled scan step
  constexpr int UF = (LF + L - 1) / L;      // f coefficients per lane
  constexpr int UE0 = (2 * N * kExtremaQD + L - 1) / L;
  constexpr int UE = UE0 < 8 ? UE0 : 8;     // staged entries per lane and round of loads
  extern __shared__ __attribute__((aligned(16))) double xlds[];
  const int tid = threadIdx.x;
  const int lane = tid % L, grp = tid / L;  // the group of L lanes owns one (trajectory, segment)
  const int ngrp = tpb * K;                 // groups of the block
  const int bl = grp / K, i = grp - bl * K;
  const int64_t b = (int64_t)blockIdx.x * tpb + bl;
  const bool active = grp < ngrp && b < B;
  const int nd = N - k;  // p^(k) coefficient count
  const int ndim = __builtin_popcount(dims);
  const int GS = extrema_group_doubles(N, qd);
  Ext* smin = reinterpret_cast<Ext*>(xlds + (size_t)ngrp * GS);
  Ext* smax = smin + ngrp;
  const int g = grp < ngrp ? grp : 0;
  double* gf = xlds + (size_t)g * GS;  // this group's f, then q, then the padded q1
  double* gq = gf + 2 * N;
  double* gq1 = gq + qd * N;  // q1_c starts at gq1 + (2c + 1) N

  Ext lo{0.0, DBL_MAX, 0x7fffffff}, hi{0.0, -DBL_MAX, 0x7fffffff};
  const int64_t bb = active ? b : 0;
  const int ii = active ? i : 0;
  const double T = times[bb * K + ii];
  const double* cs = coeffs + ((bb * K + ii) * D) * N;
  if (grp < ngrp)  // the zero pads (never overwritten)
    for (int e = lane; e < (qd + 1) * N; e += L) gq1[(e / N) * 2 * N + e % N] = 0.0;
  // ---- stage q, q1 of qd selected dimensions at a time; lane l forms f[n], n = l, l + L, ...
  double facc[UF];
#pragma unroll
  for (int u = 0; u < UF; ++u) facc[u] = 0.0;
  for (int m0 = 0; m0 < ndim; m0 += qd) {
    const int nc = ndim - m0 < qd ? ndim - m0 : qd;
    for (int e0 = 0; e0 < 2 * N * qd; e0 += UE * L) {  // (one round for L >= 8)
      double sv[UE];
      int se[UE];
#pragma unroll
      for (int u = 0; u < UE; ++u) {  // one batch of loads: entry e = (c, j): q (j < N) or q1 (j >= N)
        const int e = e0 + lane + u * L;
        const int c = e / (2 * N), j = e - c * (2 * N);
        double v = 0.0;
        if (c < nc) {
          const int d = sel_dim(dims, m0 + c);
          const int jj = j < N ? j : j - N, kk = j < N ? k : k + 1;
          if (jj + kk < N) v = cs[d * N + jj + kk] * c_ff.v[jj + kk][kk];
        }
        sv[u] = v;
        se[u] = e < 2 * N * qd ? (j < N ? c * N + j : qd * N + (2 * c + 1) * N + (j - N)) : -1;
      }
#pragma unroll
      for (int u = 0; u < UE; ++u)
        if (se[u] >= 0 && grp < ngrp) gq[se[u]] = sv[u];
    }
    lds_fence();  // (the group is L consecutive lanes of one wave)
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      const int n = lane + u * L;
      if (n >= LF) continue;
      if (ndim == 1) {  // one dimension: the roots of p^(k+1) (segment.cpp:124-130); (n >= N: a pad)
        facc[u] = gq1[N + n];
      } else {  // convolve(d, dd) (polynomial.h convolve), summed over dimensions
        double t = 0.0;
        for (int c = 0; c < nc; ++c) {
          const double* q1n = gq1 + (2 * c + 1) * N + n;  // q1_c[n - a] = q1n[-a] (pads: 0)
#pragma unroll
          for (int a = 0; a < N; ++a) t += gq[c * N + a] * q1n[-a];
        }
        facc[u] += t;
      }
    }
    if (m0 + qd < ndim) lds_fence();  // (read before the next pass overwrites q, q1)
  }
#pragma unroll
  for (int u = 0; u < UF; ++u) {
    const int n = lane + u * L;
    if (n < LF && grp < ngrp) gf[n] = facc[u];
  }
  lds_fence();
  double f[LF];
#pragma unroll
  for (int j = 0; j < LF; ++j) f[j] = gf[j];

  if (active) {
    const bool staged = ndim <= qd;  // q of every selected dimension is in LDS
    auto mag = [&](double t) {
      double s = 0.0;
      if (staged) {
        for (int c = 0; c < ndim; ++c) {
          double acc = 0.0;
#pragma unroll
          for (int j = N - 1; j >= 0; --j) acc = acc * t + gq[c * N + j];
          s += acc * acc;
        }
      } else {
        for (int d = 0; d < D; ++d) {
          if (!((dims >> d) & 1u)) continue;
          double qv[N];
#pragma unroll
          for (int j = 0; j < N; ++j) qv[j] = j < nd ? cs[d * N + j + k] * c_ff.v[j + k][k] : 0.0;
          double acc = 0.0;
#pragma unroll
          for (int j = N - 1; j >= 0; --j) acc = acc * t + qv[j];
          s += acc * acc;
        }
      }
      return sqrt(s);
    };
    const double h = T / kExtremaSamples;
    const int s0 = lane * SPL;
    double fa = horner<LF>(f, s0 * h);
    // the end points t = 0 (ord 0, lane 0) and t = T (ord 1, lane L - 1), in one pass of the wave.
    // (An exact zero of f at t = 0 or t = T is the same candidate with a later order: never chosen.)
    if (lane == 0 || lane == L - 1) {
      const double te = lane == 0 ? 0.0 : T;
      const Ext e{te, mag(te), lane == 0 ? 0 : 1};
      lo = hi = e;
    }
    for (int ch = 0; ch < SPL / CH; ++ch) {  // (one mask for L >= 4)
      const int sc = s0 + ch * CH;  // this mask's samples sc + 1 .. sc + CH
      uint64_t pend = 0;
#pragma nounroll
      for (int q0 = 0; q0 < CH; q0 += CS) {
#pragma unroll
        for (int q = 0; q < CS; ++q) {
          const int s = sc + 1 + q0 + q;
          const double tb = s == kExtremaSamples ? T : s * h;
          const double fb = horner<LF>(f, tb);
          const bool hit = fb == 0.0 || (fa < 0.0 && fb > 0.0) || (fa > 0.0 && fb < 0.0);
          pend |= hit ? 1ull << (q0 + q) : 0ull;
          fa = fb;
        }
      }
      // the candidates, lowest bit first, one per lane per round
      while (__builtin_amdgcn_ballot_w64(pend != 0) != 0) {
        if (pend != 0) {
          const int q = __builtin_ctzll(pend);
          pend &= pend - 1;
          const int s = sc + 1 + q;
          const double tb = s == kExtremaSamples ? T : s * h;
          const double tl = (s - 1) * h;
          const double fl = horner<LF>(f, tl), fb = horner<LF>(f, tb);
          const double t = fb == 0.0 ? tb : refine<LF>(f, tl, tb, fl, fb);
          const Ext e{t, mag(t), 2 + s};
          if (better_max(e, hi)) hi = e;
          if (better_min(e, lo)) lo = e;
        }
      }
    }
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

// lanes per segment and trajectories per block: 8 lanes while a trajectory fits a block (K <= 64),
// then fewer; the trajectories per block that keep the block's waves fullest (K = 10: 8 lanes, 4
// trajectories, 320 threads = 5 full waves).  (Config 2, same box: 16 lanes 0.130 ms, 8 lanes 0.104,
// 4 lanes 0.106 -- fewer lanes share the per-segment work of forming f over fewer waves, more
// lanes scan fewer samples each.)
void extrema_geometry(int K, int* lanes, int* tpb, int* threads) {
  int L = 8;
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
  // dimensions staged per pass: as many as the selection needs (at most 4) while the block's LDS
  // stays within kMaxLdsPerBlock, at least 1
  const int ndim = __builtin_popcount(dims);
  auto bytes = [&](int qd) {
    return sizeof(double) * (size_t)tpb * K * extrema_group_doubles(N, qd) + 2 * sizeof(Ext) * (size_t)tpb * K;
  };
  int qd = ndim < kExtremaQD ? ndim : kExtremaQD;
  while (qd > 1 && bytes(qd) > kMaxLdsPerBlock) --qd;
  const size_t lds = bytes(qd);
  if (lds > kMaxLdsHard) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((B + tpb - 1) / tpb)), block(threads);
  launch_kernel((min_max_magnitude_kernel<N, L>), grid, block, (uint32_t)lds, stream, coeffs, times, B, K, D, k, dims,
                tpb, qd, mn, mx);
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
