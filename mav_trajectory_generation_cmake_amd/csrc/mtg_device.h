// mtg_device.h -- device helpers shared by the solve kernels (mtg_kernels.hip: general
// LDS-resident kernel; mtg_solve_reg.hip: register-resident kernel for K <= 12, N = 12 to K = 20).
#pragma once

#include <float.h>

#include "mtg.h"
#include "mtg_internal.h"
#include "mtg_tables.inc"

namespace mtg {

// Exact-rational constant tables (gen_tables.py), one copy per translation unit:
//   A(1)^-1                          the mapping-matrix inverse at T = 1 (lin_impl:133-169)
//   Htilde(N, r) = A(1)^-T Q(1) A(1)^-1   Q with the reference's factor 2 (lin_impl:574-589)
static __constant__ double c_a1inv[MTG_A1INV_SIZE] = {MTG_A1INV_VALUES};
static __constant__ double c_htilde[MTG_HTILDE_SIZE] = {MTG_HTILDE_VALUES};
static __constant__ double c_hbl[MTG_HBL_SIZE] = {MTG_HBL_VALUES};  // BL block of Htilde, contiguous

// Block of 64 threads = one wave; all LDS traffic is intra-wave.
constexpr int kBlock = 64;
constexpr size_t kMaxLdsPerBlock = 64 * 1024;
constexpr size_t kMaxLdsHard = 160 * 1024;

// Orders this wave's LDS accesses (every block is one wave): waits for its LDS operations only,
// and is a compiler memory barrier.  __syncthreads() would also wait for the wave's outstanding
// global stores (vmcnt counts stores on gfx9), which in a store-per-round epilogue exposes the
// HBM write latency once per round.
__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// A buffer resource over [base, base + bytes), built from wave-uniform values (readfirstlane, so the
// compiler keeps it in SGPRs and emits no waterfall loop around the buffer instructions).  Loads and
// stores address it with 32-bit per-lane byte offsets; a store whose offset is past `bytes` is
// dropped by the hardware, which is how a lane skips a store without a branch.
constexpr uint32_t kBufOOB = 0x80000000u;  // an offset past any resource this code builds
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  void* q = reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// Native 2 x f64 vector (HIP's double2 is a struct: arrays of it in registers can fall back to
// private memory where a vector type stays in VGPRs).
typedef double dvec2 __attribute__((ext_vector_type(2)));

// Streaming (nontemporal) 16-B store of write-once output: `global_store_dwordx4 ... nt`.  The
// coefficients are never re-read by the kernel; with plain stores they sat dirty in the XCDs' L2s
// and drained at the end of the launch (config 2, B = 1e4: 18.8 -> 17.6 us with nt).
__device__ __forceinline__ void store_stream(double2* dst, const double2& v) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store(d2v{v.x, v.y}, reinterpret_cast<d2v*>(dst));
}

// 1/x from v_rcp_f64 plus two Newton steps (full FP64 accuracy; no IEEE division sequence).
__device__ __forceinline__ double rcp(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-x, y, 1.0);
  return __builtin_fma(y, e, y);
}

// s[k] = T^k (k < H) and sc = T^(1-2R) = 1 / (T^R T^(R-1)): the time-scaling of one segment.
template <int H, int R>
__device__ __forceinline__ void seg_powers(double T, double (&s)[H], double& sc) {
  static_assert(R >= 0 && R < H, "derivative_to_optimize must be in [0, N/2-1]");
  s[0] = 1.0;
#pragma unroll
  for (int k = 1; k < H; ++k) s[k] = s[k - 1] * T;
  if constexpr (R == 0) {
    sc = T;
  } else {
    sc = rcp(s[R] * s[R - 1]);
  }
}

// Status bits of one segment time.  T must be > 0 and finite (CHECK_GT(segment_time, 0), lin_impl:287):
// otherwise BAD_TIME.  For 0 < T < DBL_EPSILON the reference's baseCoeffsWithTime keeps only the
// t = 0 entry (polynomial.h:225), so its mapping matrix A(T) is singular and its solve is not
// defined: reported as NOT_SPD, not as a bad time.
__device__ __forceinline__ int time_bits(double T) {
  return !(T > 0.0 && T <= DBL_MAX) ? MTG_TRAJ_BAD_TIME : (T < DBL_EPSILON ? MTG_TRAJ_NOT_SPD : 0);
}

template <int H>
__device__ __forceinline__ void load_fixed(const double* vals, int v, int D, int d, unsigned m,
                                           double (&x)[H]) {
  const double* p = vals + ((size_t)v * H) * D + d;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const double t = p[k * D];
    x[k] = ((m >> k) & 1u) ? t : 0.0;
  }
}

// Running minimum of the LDL^T pivots in which a NaN pivot sticks (NOT_SPD is reported for a
// minimum <= 0 or not finite): v_min_f64 returns the other operand for a quiet NaN, so a NaN pivot
// is folded in as -inf.  Two VALU operations (compare-unordered + select folds into the min's
// operand) instead of a compare/compare/or/select pair.
__device__ __forceinline__ double pivot_min(double pmin, double dj) {
  return __builtin_fmin(pmin, dj != dj ? -__builtin_inf() : dj);
}

// S = L diag(d) L^T (L unit lower, below the diagonal of S; only the lower triangle of S is
// read); dinv = 1/d.  Returns the smallest pivot (<= 0 or non-finite: R_pp is not SPD; the
// reference never checks, lin_impl:355-368).
template <int H>
__device__ __forceinline__ double ldlt(double (&S)[H][H], double (&dinv)[H]) {
  double pmin = DBL_MAX;
  double dg[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    double w[H];
    double dj = S[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) {
      w[k] = S[j][k] * dg[k];
      dj -= S[j][k] * w[k];
    }
    pmin = (dj < pmin || dj != dj) ? dj : pmin;  // a NaN pivot sticks (NOT_SPD)
    const double inv = rcp(dj);
    dg[j] = dj;
    dinv[j] = inv;
#pragma unroll
    for (int i = j + 1; i < H; ++i) {
      double t = S[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= S[i][k] * w[k];
      S[i][j] = t * inv;
    }
  }
  return pmin;
}

// x = S^-1 b with S factored in place by ldlt()
template <int H>
__device__ __forceinline__ void ldlt_solve(const double (&S)[H][H], const double (&dinv)[H],
                                           const double (&b)[H], double (&x)[H]) {
  double y[H];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    double t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t -= S[i][k] * y[k];
    y[i] = t;
  }
#pragma unroll
  for (int i = H - 1; i >= 0; --i) {
    double t = y[i] * dinv[i];
#pragma unroll
    for (int k = i + 1; k < H; ++k) t -= S[k][i] * x[k];
    x[i] = t;
  }
}

// Per-trajectory LDS slot (doubles): exchange buffer (LG x h), G_v (K x h x h), Z_v (V x D x h:
// z_v after the forward sweep, the pinned solution x_v after the backward sweep).
__host__ __device__ __forceinline__ int slot_doubles(int H, int D, int K, int LG) {
  return LG * H + K * H * H + (K + 1) * D * H;
}

// Re-materialise a uniform table pointer inside a loop so the compiler reloads the table
// from the scalar cache instead of hoisting 100+ doubles into SGPRs and spilling them.
typedef const __attribute__((address_space(4))) double cdouble;
__device__ __forceinline__ cdouble* launder(const double* p) {
  cdouble* q = (cdouble*)p;
  asm volatile("" : "+s"(q));
  return q;
}

}  // namespace mtg
