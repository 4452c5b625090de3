// mtg_vertex.hip -- the two maps between a trajectory's vertex derivatives and its coefficients,
// batched:
//
// * coefficients_from_vertices: c_i = A(T_i)^-1 [x_i; x_{i+1}] per (segment, dimension), the
//   reference's updateSegmentsFromCompactConstraints (lin_impl:253-273) after
//   setFreeConstraints (polynomial_optimization_linear.h:185-186) -- every vertex derivative
//   (fixed and free) is given, nothing is solved.  Same arithmetic as the solve kernels'
//   epilogue: A(T)^-1 = diag(T^-j) A(1)^-1 S(T) from the exact-rational A(1)^-1 table, with the
//   segment's start position subtracted first (only c_0 changes; no cancellation of p_i
//   against p_{i+1} in c_j, j >= h).
// * vertex_derivatives: the reference's M^+ A p (nl_impl:162-180, used by
//   computeInitialSolutionWithoutPositionConstraints): the end derivatives A_i c_i of every
//   segment, mapped to the (vertex, derivative) unknowns by the pseudo-inverse of the 0/1
//   reordering matrix M (lin_impl:172-250), i.e. the mean of the two segment ends that meet at an
//   interior vertex and the single end at the first / last vertex.
//
// Both are HBM-bound streams.  A block of 256 threads owns TB consecutive trajectories: it
// stages their input (contiguous in HBM) into LDS with coalesced loads, computes one item per
// thread out of LDS, writes the results into LDS and stores them as one contiguous run.
#include "mtg_device.h"

namespace mtg {

constexpr int kVtxThreads = 256;

namespace {

// dst[i] = src[i] for i < n by the block, U loads per thread in flight before the stores.
template <int U>
__device__ __forceinline__ void stage_copy(const double* __restrict__ src, double* dst, int n, int tid) {
  for (int base = 0; base < n; base += U * kVtxThreads) {
    double r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * kVtxThreads + tid;
      r[u] = src[i < n ? i : n - 1];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * kVtxThreads + tid;
      if (i < n) dst[i] = r[u];
    }
  }
}

// falling factorial k!/(k-n)! (Polynomial::base_coefficients_, src/polynomial.cpp:140-155)
__device__ __forceinline__ double falling(int k, int n) {
  double f = 1.0;
  for (int q = 0; q < n; ++q) f *= (double)(k - q);
  return f;
}

// vertex values [TB][V][H][D] -> coefficients [TB][K][D][N]
template <int N>
__global__ __launch_bounds__(kVtxThreads) void coefficients_from_vertices_kernel(const double* __restrict__ values,
                                                                                 const double* __restrict__ times,
                                                                                 double* __restrict__ coeffs,
                                                                                 int64_t B, int K, int D, int TB) {
  constexpr int H = N / 2;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int V = K + 1, xsz = V * H * D, csz = K * D * N;
  const int64_t b0 = (int64_t)blockIdx.x * TB;
  const int nb = (int)(B - b0 < TB ? B - b0 : TB);
  double* xv = lds;                // [nb][V][H][D]
  double* tl = xv + TB * xsz;      // [nb][K]
  double* co = tl + TB * K;        // [nb][K][D][N] (TB * K even: 16-B aligned when TB even)
  const int tid = threadIdx.x;
  stage_copy<8>(values + b0 * xsz, xv, nb * xsz, tid);
  stage_copy<2>(times + b0 * K, tl, nb * K, tid);
  __syncthreads();
  const double* Ai1 = c_a1inv + MTG_A1INV_OFF(N);
  for (int it = tid; it < nb * K * D; it += kVtxThreads) {
    const int bl = it / (K * D), rem = it - bl * (K * D), i = rem / D, d = rem - i * D;
    const double T = tl[bl * K + i];
    const double* x = xv + bl * xsz;
    double s[H];
    s[0] = 1.0;
#pragma unroll
    for (int k = 1; k < H; ++k) s[k] = s[k - 1] * T;
    double sh[N];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      sh[k] = s[k] * x[(i * H + k) * D + d];
      sh[H + k] = s[k] * x[((i + 1) * H + k) * D + d];
    }
    const double p0 = sh[0];
    sh[0] = 0.0;
    sh[H] -= p0;
    const double tinv = rcp(T);
    double tp = 1.0;
    double* out = co + (size_t)it * N;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double acc;
      if (j < H) {
        acc = (j == 0) ? p0 : Ai1[j * N + j] * sh[j];
      } else {
        acc = 0.0;
#pragma unroll
        for (int q = 1; q < N; ++q) acc += Ai1[j * N + q] * sh[q];
      }
      out[j] = acc * tp;
      tp *= tinv;
    }
  }
  __syncthreads();
  double* dst = coeffs + b0 * csz;
  for (int e = tid; e < nb * csz; e += kVtxThreads) dst[e] = co[e];
}

// coefficients [TB][K][D][N] -> vertex values [TB][V][H][D]
template <int N>
__global__ __launch_bounds__(kVtxThreads) void vertex_derivatives_kernel(const double* __restrict__ coeffs,
                                                                         const double* __restrict__ times,
                                                                         double* __restrict__ values, int64_t B,
                                                                         int K, int D, int TB) {
  constexpr int H = N / 2;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int V = K + 1, xsz = V * H * D, csz = K * D * N;
  const int64_t b0 = (int64_t)blockIdx.x * TB;
  const int nb = (int)(B - b0 < TB ? B - b0 : TB);
  double* co = lds;                // [nb][K][D][N]
  double* tl = co + TB * csz;      // [nb][K]
  double* xv = tl + TB * K;        // [nb][V][H][D]
  const int tid = threadIdx.x;
  stage_copy<8>(coeffs + b0 * csz, co, nb * csz, tid);
  stage_copy<2>(times + b0 * K, tl, nb * K, tid);
  __syncthreads();
  // item (trajectory, vertex, derivative, dimension) in output order
  for (int it = tid; it < nb * xsz; it += kVtxThreads) {
    const int bl = it / xsz, rem = it - bl * xsz;
    const int v = rem / (H * D), r2 = rem - v * (H * D), k = r2 / D, d = r2 - k * D;
    double sum = 0.0;
    int cnt = 0;
    if (v < K) {  // start of segment v: p^(k)(0) = k! c_k
      sum += falling(k, k) * co[((bl * K + v) * D + d) * N + k];
      ++cnt;
    }
    if (v > 0) {  // end of segment v-1: p^(k)(T) = sum_j j!/(j-k)! c_j T^(j-k)  (Horner)
      const double T = tl[bl * K + v - 1];
      const double* c = co + ((bl * K + v - 1) * D + d) * N;
      double acc = 0.0;
      for (int j = N - 1; j >= k; --j) acc = acc * T + falling(j, k) * c[j];
      sum += acc;
      ++cnt;
    }
    xv[it] = cnt == 2 ? 0.5 * sum : sum;
  }
  __syncthreads();
  double* dst = values + b0 * xsz;
  for (int e = tid; e < nb * xsz; e += kVtxThreads) dst[e] = xv[e];
}

int traj_per_block(int N, int D, int K) {
  const int H = N / 2, V = K + 1;
  const size_t per = sizeof(double) * ((size_t)V * H * D + K + (size_t)K * D * N);
  int tb = (int)(48 * 1024 / per);
  if (tb > 16) tb = 16;
  return tb & ~1;  // even: the LDS regions stay 16-B aligned
}

template <int N>
hipError_t launch_vertex_n(bool to_coeffs, const double* in, const double* times, double* out, int64_t B, int K,
                           int D, hipStream_t stream) {
  const int tb = traj_per_block(N, D, K);
  if (tb < 2) return hipErrorInvalidValue;
  if (B == 0) return hipSuccess;
  const int H = N / 2, V = K + 1;
  const size_t lds = sizeof(double) * (size_t)tb * ((size_t)V * H * D + K + (size_t)K * D * N);
  const dim3 grid((unsigned)((B + tb - 1) / tb)), block(kVtxThreads);
  if (to_coeffs)
    launch_kernel((coefficients_from_vertices_kernel<N>), grid, block, lds, stream, in, times, out, B, K, D, tb);
  else
    launch_kernel((vertex_derivatives_kernel<N>), grid, block, lds, stream, in, times, out, B, K, D, tb);
  return hipGetLastError();
}

}  // namespace

bool vertex_map_fits(int N, int D, int K) { return traj_per_block(N, D, K) >= 2; }

hipError_t launch_vertex_map(bool to_coeffs, int N, const double* in, const double* times, double* out, int64_t B,
                             int K, int D, hipStream_t stream) {
  switch (N) {
    case 2: return launch_vertex_n<2>(to_coeffs, in, times, out, B, K, D, stream);
    case 4: return launch_vertex_n<4>(to_coeffs, in, times, out, B, K, D, stream);
    case 6: return launch_vertex_n<6>(to_coeffs, in, times, out, B, K, D, stream);
    case 8: return launch_vertex_n<8>(to_coeffs, in, times, out, B, K, D, stream);
    case 10: return launch_vertex_n<10>(to_coeffs, in, times, out, B, K, D, stream);
    case 12: return launch_vertex_n<12>(to_coeffs, in, times, out, B, K, D, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
