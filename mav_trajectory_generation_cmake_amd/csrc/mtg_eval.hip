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

// Samples per chunk (one wave: lane l evaluates sample 64 c + l) and chunks checkpointed per round.
constexpr int kChunk = 64;
constexpr int kRoundChunks = 256;
constexpr int kEvalThreads = 256;

// One workgroup per trajectory.  Lane 0 replays the reference's clock (exactly the recurrence
// above) and checkpoints (acc, tin, segment) at every 64th sample into LDS; then every lane
// replays at most 63 steps from its chunk's checkpoint -- the same floating-point operations in
// the same order, so sample times and segment choices stay bit-identical -- and evaluates its
// sample.  The trajectory's coefficients are staged in LDS; output rows are contiguous per wave.
template <int N>
__global__ __launch_bounds__(kEvalThreads) void eval_range_kernel(int D, int K, const double* coeffs,
                                                                  const double* times, double t_start, double dt,
                                                                  int derivative, const int64_t* counts,
                                                                  const int64_t* offsets, double* out,
                                                                  double* sample_times) {
  // HIP defaults to -ffp-contract=fast-honor-pragmas: without this pragma the Horner step below
  // becomes an FMA (v_fmac_f64) and differs from the reference in the last bit.
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t n_total = counts[b];
  if (n_total <= 0) return;
  double* cf = lds;                               // [K][D][N]
  double* tl = cf + K * D * N;                    // [K]
  double* ck_acc = tl + K;                        // [kRoundChunks]
  double* ck_tin = ck_acc + kRoundChunks;         // [kRoundChunks]
  int* ck_seg = reinterpret_cast<int*>(ck_tin + kRoundChunks);
  const double* cb = coeffs + b * (int64_t)K * D * N;
  for (int i = tid; i < K * D * N; i += kEvalThreads) cf[i] = cb[i];
  for (int i = tid; i < K; i += kEvalThreads) tl[i] = times[b * K + i];
  double row[N];
#pragma unroll
  for (int j = 0; j < N; ++j) row[j] = base_coeff(derivative, j);
  const int64_t base = offsets[b];
  // lane 0's running clock (state before the switch check of sample n)
  int seg = 0;
  double acc = 0.0, tin = 0.0;
  if (tid == 0) range_start(times + b * K, K, t_start, &seg, &acc, &tin);
  __syncthreads();
  const int wave = tid / kChunk, lane = tid % kChunk;
  for (int64_t n0 = 0; n0 < n_total; n0 += (int64_t)kRoundChunks * kChunk) {
    const int64_t left = n_total - n0;
    const int nch = (int)((left + kChunk - 1) / kChunk < kRoundChunks ? (left + kChunk - 1) / kChunk : kRoundChunks);
    if (tid == 0) {
      for (int c = 0; c < nch; ++c) {
        ck_acc[c] = acc;
        ck_tin[c] = tin;
        ck_seg[c] = seg;
        for (int s = 0; s < kChunk; ++s) {  // advance one chunk: 64 emitted samples
          while (tin > tl[seg] && seg < K - 1) {
            tin = tin - tl[seg];
            ++seg;
          }
          tin += dt;
          acc += dt;
        }
      }
    }
    __syncthreads();
    for (int c = wave; c < nch; c += kEvalThreads / kChunk) {
      const int64_t n = n0 + (int64_t)c * kChunk + lane;
      double a = ck_acc[c], t = ck_tin[c];
      int i = ck_seg[c];
      for (int s = 0;; ++s) {
        while (t > tl[i] && i < K - 1) {
          t = t - tl[i];
          ++i;
        }
        if (s == lane) break;
        t += dt;
        a += dt;
      }
      if (n < n_total) {
        const double* cs = cf + (i * D) * N;
        for (int d = 0; d < D; ++d) {
          double v = 0.0;
          if (derivative < N) {
            const double* c = cs + d * N;
            v = row[N - 1] * c[N - 1];
#pragma unroll
            for (int j = N - 2; j >= 0; --j) {
              if (j >= derivative) {
                v = v * t;
                v = v + row[j] * c[j];
              }
            }
          }
          out[(base + n) * D + d] = v;
        }
        if (sample_times) sample_times[base + n] = a;
      }
    }
    __syncthreads();
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
                             double t_start, double t_end, double dt, int derivative, const int64_t* counts,
                             const int64_t* offsets, double* out, double* sample_times, hipStream_t stream) {
  (void)t_end;  // the sample counts (eval_count_kernel) already encode t_end
  if (B == 0) return hipSuccess;
  const size_t lds = sizeof(double) * ((size_t)K * D * N + K + 2 * kRoundChunks) + sizeof(int) * kRoundChunks;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
#define MTG_EVAL_CASE(NN)                                                                               \
  case NN:                                                                                              \
    hipLaunchKernelGGL(eval_range_kernel<NN>, dim3((unsigned)B), dim3(kEvalThreads), lds, stream, D, K, \
                       coeffs, times, t_start, dt, derivative, counts, offsets, out, sample_times);     \
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
