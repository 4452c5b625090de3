// mtg_eval.hip -- batched Trajectory::evaluateRange (src/trajectory.cpp:68-128).
//
// The reference advances its clock by repeated FP addition (acc += dt,
// tin += dt, tin -= T_i at a segment switch, :109-126), so the number of
// samples and every sample time depend on the sequential rounding.  These
// kernels replay exactly that recurrence per trajectory (bit-identical sample
// times and counts) and evaluate the segment polynomials with the
// reference's Horner form (Polynomial::evaluate, polynomial.h:138-151).
#include <float.h>

#include "mtg_internal.h"
#include "mtg_tables.inc"

namespace mtg {

// Polynomial::base_coefficients_(n, i) = i!/(i-n)! (src/polynomial.cpp:140-155)
__device__ __forceinline__ double base_coeff(int n, int i) {
  if (i < n) return 0.0;
  double out = 1.0;
  for (int k = i - n + 1; k <= i; ++k) out *= (double)k;
  return out;
}

// Locate the start segment exactly as :82-105; returns false if t_start is out of range.
__device__ __forceinline__ bool range_start(const double* tms, int K, double t_start, int* seg,
                                            double* acc, double* tin) {
  double a = 0.0;
  int i = 0;
  for (i = 0; i < K; ++i) {
    a += tms[i];
    if (a > t_start) break;
  }
  if (t_start > a) return false;
  if (i >= K) i = K - 1;  // reference indexes segments_[K] here (UB); clamp to the last segment
  a -= tms[i];
  *seg = i;
  *acc = a;
  *tin = t_start - a;
  return true;
}

__global__ void eval_count_kernel(int K, int64_t B, const double* times, double t_start, double t_end,
                                  double dt, int64_t* counts) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* tms = times + b * K;
  int i;
  double acc, tin;
  int64_t n = 0;
  if (range_start(tms, K, t_start, &i, &acc, &tin)) {
    while (acc < t_end) {
      if (tin > tms[i]) {
        tin = tin - tms[i];
        if (++i >= K) break;
        continue;
      }
      ++n;
      tin += dt;
      acc += dt;
    }
  }
  counts[b] = n;
}

template <int N>
__global__ void eval_range_kernel(int D, int K, int64_t B, const double* coeffs, const double* times,
                                  double t_start, double t_end, double dt, int derivative,
                                  const int64_t* offsets, double* out, double* sample_times) {
  // HIP defaults to -ffp-contract=fast-honor-pragmas: without this pragma the Horner step below
  // becomes an FMA (v_fmac_f64) and differs from the reference in the last bit.
#pragma clang fp contract(off)
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const double* tms = times + b * K;
  const double* cb = coeffs + b * (int64_t)K * D * N;
  double row[N];
#pragma unroll
  for (int j = 0; j < N; ++j) row[j] = base_coeff(derivative, j);
  int i;
  double acc, tin;
  if (!range_start(tms, K, t_start, &i, &acc, &tin)) return;
  int64_t n = offsets[b];
  while (acc < t_end) {
    if (tin > tms[i]) {
      tin = tin - tms[i];
      if (++i >= K) break;
      continue;
    }
    const double* cs = cb + (int64_t)i * D * N;
    for (int d = 0; d < D; ++d) {
      double v = 0.0;
      if (derivative < N) {
        const double* c = cs + d * N;
        // result = row[N-1] c[N-1]; result *= t; result += row[j] c[j]: plain operators under
        // the contract(off) pragma above, so the rounding is the reference's multiply-then-add
        // (the pragma does not reach into inlined helpers such as __dmul_rn)
        v = row[N - 1] * c[N - 1];
#pragma unroll
        for (int j = N - 2; j >= 0; --j) {
          if (j >= derivative) {
            v = v * tin;
            v = v + row[j] * c[j];
          }
        }
      }
      out[n * D + d] = v;
    }
    if (sample_times) sample_times[n] = acc;
    ++n;
    tin += dt;
    acc += dt;
  }
}

hipError_t launch_eval_count(int N, int D, int K, int64_t B, const double* times, double t_start,
                             double t_end, double dt, int64_t* counts, hipStream_t stream) {
  (void)N;
  (void)D;
  const int block = 256;
  const int64_t grid = (B + block - 1) / block;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(eval_count_kernel, dim3((unsigned)grid), dim3(block), 0, stream, K, B, times, t_start,
                     t_end, dt, counts);
  return hipGetLastError();
}

hipError_t launch_eval_range(int N, int D, int K, int64_t B, const double* coeffs, const double* times,
                             double t_start, double t_end, double dt, int derivative,
                             const int64_t* offsets, double* out, double* sample_times, hipStream_t stream) {
  const int block = 64;
  const int64_t grid = (B + block - 1) / block;
  if (grid == 0) return hipSuccess;
#define MTG_EVAL_CASE(NN)                                                                          \
  case NN:                                                                                         \
    hipLaunchKernelGGL(eval_range_kernel<NN>, dim3((unsigned)grid), dim3(block), 0, stream, D, K, B, \
                       coeffs, times, t_start, t_end, dt, derivative, offsets, out, sample_times); \
    break;
  switch (N) {
    MTG_EVAL_CASE(2)
    MTG_EVAL_CASE(4)
    MTG_EVAL_CASE(6)
    MTG_EVAL_CASE(8)
    MTG_EVAL_CASE(10)
    MTG_EVAL_CASE(12)
    default: return hipErrorInvalidValue;
  }
#undef MTG_EVAL_CASE
  return hipGetLastError();
}

}  // namespace mtg
