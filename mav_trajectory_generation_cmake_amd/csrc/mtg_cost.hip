// mtg_cost.hip -- cost and gradient of fixed vertex derivatives at candidate segment times
// (mtg_cost_at_times_batch): the reference's getCostAndGradientDerivative
// (polynomial_optimization_nonlinear_impl.h:1452-1520) evaluated at the perturbed times of its
// numerical time gradient (getCostAndGradientTime, :2153-2238).
//
// For segment i, dimension d and end values x = [x_i; x_{i+1}] (2h derivatives), the reference's
// d^T R d restricted to the segment is x^T A^-T Q A^-1 x = T^(1-2r) (S x)^T Htilde (S x),
// S = diag(T^(p mod h)).  At fixed x this is T^(1-2r) sum_m a_m T^m with
//   a_m = sum over (p, q) with (p mod h) + (q mod h) = m of Htilde_pq x_p x_q,   m = 0 .. 2h-2,
// so each (segment, dimension) column costs one O(N^2) reduction, shared by all candidates, and
// each candidate a degree-(2h-2) Horner evaluation -- instead of an N x N mat-vec per candidate.
// (For r >= 1 the positions are first made relative to x_i[0]: Htilde annihilates a common
// position offset, so the value is unchanged and the cancellation on short segments is gone.)
//
// The gradient 2 (R(T_c) d)_free needs Htilde (S x) per candidate; it is formed per lane (one lane
// per candidate) with Htilde from the scalar cache, and written in the reference's free order.
//
// Mapping: one wave per trajectory; LDS holds the trajectory's polynomial coefficients
// [K*D][2h-1], the segment times and its vertex values; lane c serves candidates c, c+64, ...
#include "mtg_device.h"

namespace mtg {

struct CostArgs {
  const double* values;  // [B][V][h][D] all derivatives
  const uint8_t* mask;   // [B][V] (gradient only)
  const double* times;   // [B][K]
  const double* scales;  // [C][K]
  double* cost;          // [B][C]
  double* grad;          // [B][C][D][V*h] (nullable)
  int64_t B;
  int K, D, C;
};

namespace {

template <int N, int R>
__global__ __launch_bounds__(64) void cost_at_times_kernel(CostArgs a) {
  constexpr int H = N / 2;
  constexpr int M = 2 * H - 1;
  constexpr unsigned HM = (1u << H) - 1u;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int K = a.K, V = K + 1, D = a.D, C = a.C;
  const int cols = K * D;
  double* am = lds;                  // [cols][M]
  double* tl = am + cols * M;        // [K]
  double* xv = tl + K;               // [V][H][D]
  const double* vals = a.values + b * (int64_t)V * H * D;
  for (int i = lane; i < V * H * D; i += 64) xv[i] = vals[i];
  for (int i = lane; i < K; i += 64) tl[i] = a.times[b * K + i];
  __syncthreads();

  cdouble* Ht = (cdouble*)(c_htilde + MTG_HTILDE_OFF(N, R));
  // ---- per (segment, dimension) column: the coefficients a_m of the cost polynomial in T
  for (int j = lane; j < cols; j += 64) {
    const int i = j / D, d = j - i * D;
    double x[N];
#pragma unroll
    for (int k = 0; k < H; ++k) x[k] = xv[(i * H + k) * D + d], x[H + k] = xv[((i + 1) * H + k) * D + d];
    if (R >= 1) {
      x[H] -= x[0];
      x[0] = 0.0;
    }
    double c[M];
#pragma unroll
    for (int m = 0; m < M; ++m) c[m] = 0.0;
#pragma unroll
    for (int p = 0; p < N; ++p) {
      c[2 * (p % H)] += Ht[p * N + p] * x[p] * x[p];
#pragma unroll
      for (int q = p + 1; q < N; ++q) c[(p % H) + (q % H)] += 2.0 * Ht[p * N + q] * x[p] * x[q];
    }
#pragma unroll
    for (int m = 0; m < M; ++m) am[j * M + m] = c[m];
  }
  __syncthreads();

  // ---- candidates: J(c) = sum_i T^(1-2r) sum_d sum_m a_m T^m
  for (int cc = lane; cc < C; cc += 64) {
    const double* sc_row = a.scales + (int64_t)cc * K;
    double J = 0.0;
    for (int i = 0; i < K; ++i) {
      const double T = tl[i] * sc_row[i];
      double s[H], sc;
      seg_powers<H, R>(T, s, sc);
      double seg = 0.0;
      for (int d = 0; d < D; ++d) {
        const double* c = am + (i * D + d) * M;
        double p = c[M - 1];
#pragma unroll
        for (int m = M - 2; m >= 0; --m) p = p * T + c[m];
        seg += p;
      }
      J += sc * seg;
    }
    a.cost[b * C + cc] = J;
  }

  if (!a.grad) return;
  // ---- gradient 2 (R d)_free: vertex v collects the top rows of segment v and the bottom rows
  // of segment v-1, each 2 T^(1-2r) S (Htilde S x)
  const uint8_t* msk = a.mask + b * V;
  for (int cc = lane; cc < C; cc += 64) {
    const double* sc_row = a.scales + (int64_t)cc * K;
    for (int d = 0; d < D; ++d) {
      double* g = a.grad + ((b * C + cc) * D + d) * (int64_t)(V * H);
      double prevb[H];
#pragma unroll
      for (int k = 0; k < H; ++k) prevb[k] = 0.0;
      int idx = 0;
      for (int i = 0; i <= K; ++i) {
        double top[H], bot[H];
        if (i < K) {
          const double T = tl[i] * sc_row[i];
          double s[H], sc;
          seg_powers<H, R>(T, s, sc);
          double sh[N];
#pragma unroll
          for (int k = 0; k < H; ++k) sh[k] = s[k] * xv[(i * H + k) * D + d], sh[H + k] = s[k] * xv[((i + 1) * H + k) * D + d];
          if (R >= 1) {
            sh[H] -= sh[0];
            sh[0] = 0.0;
          }
#pragma unroll
          for (int p = 0; p < N; ++p) {
            double y = 0.0;
#pragma unroll
            for (int q = 0; q < N; ++q) y += Ht[p * N + q] * sh[q];
            const double gp = 2.0 * sc * s[p % H] * y;
            if (p < H) top[p] = gp;
            else bot[p - H] = gp;
          }
        } else {
#pragma unroll
          for (int k = 0; k < H; ++k) top[k] = 0.0, bot[k] = 0.0;
        }
        const unsigned mv = msk[i] & HM;
#pragma unroll
        for (int k = 0; k < H; ++k)
          if (!((mv >> k) & 1u)) g[idx++] = prevb[k] + top[k];
#pragma unroll
        for (int k = 0; k < H; ++k) prevb[k] = bot[k];
      }
    }
  }
}

template <int N, int R>
hipError_t launch_cost_nr(const CostArgs& a, hipStream_t stream) {
  constexpr int H = N / 2;
  const size_t lds = sizeof(double) * ((size_t)a.K * a.D * (2 * H - 1) + a.K + (size_t)(a.K + 1) * H * a.D);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  if (a.B == 0) return hipSuccess;
  launch_kernel((cost_at_times_kernel<N, R>), dim3((unsigned)a.B), dim3(64), lds, stream, a);
  return hipGetLastError();
}

template <int N>
hipError_t launch_cost_n(const CostArgs& a, int r, hipStream_t stream) {
  switch (r) {
    case 0: return launch_cost_nr<N, 0>(a, stream);
    case 1: if constexpr (N / 2 > 1) return launch_cost_nr<N, 1>(a, stream); break;
    case 2: if constexpr (N / 2 > 2) return launch_cost_nr<N, 2>(a, stream); break;
    case 3: if constexpr (N / 2 > 3) return launch_cost_nr<N, 3>(a, stream); break;
    case 4: if constexpr (N / 2 > 4) return launch_cost_nr<N, 4>(a, stream); break;
    case 5: if constexpr (N / 2 > 5) return launch_cost_nr<N, 5>(a, stream); break;
    default: break;
  }
  return hipErrorInvalidValue;
}

}  // namespace

size_t cost_lds_bytes(int N, int D, int K) {
  const int H = N / 2;
  return sizeof(double) * ((size_t)K * D * (2 * H - 1) + K + (size_t)(K + 1) * H * D);
}

hipError_t launch_cost_at_times(int N, int r, const double* values, const uint8_t* mask, const double* times,
                                const double* scales, double* cost, double* grad, int64_t B, int K, int D, int C,
                                hipStream_t stream) {
  CostArgs a{values, mask, times, scales, cost, grad, B, K, D, C};
  switch (N) {
    case 2: return launch_cost_n<2>(a, r, stream);
    case 4: return launch_cost_n<4>(a, r, stream);
    case 6: return launch_cost_n<6>(a, r, stream);
    case 8: return launch_cost_n<8>(a, r, stream);
    case 10: return launch_cost_n<10>(a, r, stream);
    case 12: return launch_cost_n<12>(a, r, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
