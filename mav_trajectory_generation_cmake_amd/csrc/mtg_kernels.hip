// mtg_kernels.hip -- hand-written HIP kernels (gfx950) of the batched
// minimum-derivative polynomial optimizer.
//
// What the reference computes per trajectory (lin_impl =
// mav_trajectory_generation/include/mav_trajectory_generation/impl/
// polynomial_optimization_linear_impl.h):
//   Q_i, A_i, A_i^-1           updateSegmentTimes        lin_impl:276-295
//   M (fixed/free reordering)  setupConstraintReorderingMatrix  :172-250
//   R = M^T blkdiag(A^-T Q A^-1) M; R_pp d_p = -R_pf d_f   solveLinear :298-369
//   c_i = A_i^-1 (M d)_i       updateSegmentsFromCompactConstraints :253-273
//   0.5 sum c^T Q c            computeCost               :114-130
//
// How this file computes the same minimiser (DESIGN.md "Algorithm"):
// * Unknowns are ordered by (vertex, derivative), exactly the reference's
//   std::set order (Constraint::operator<, polynomial_optimization_linear.h:273-280),
//   so R is block-tridiagonal with h x h blocks (h = N/2): vertex v couples
//   only to v-1 and v+1.  M is never formed: slot s of segment i is
//   (vertex i + (s >= h), derivative s mod h).
// * Fixed derivatives are eliminated by "pinning": their rows/columns of R
//   become the identity and their values move to the right-hand side, which
//   is algebraically R_pp d_p = -R_pf d_f with uniform h x h blocks for any
//   per-vertex mask (n_free == 0, lin_impl:333-339, falls out naturally).
// * Each block is rebuilt from an exact-rational constant table:
//   H_i = T^(1-2r) S Htilde S,  A_i^-1 = diag(T^-j) A(1)^-1 S,  S = diag(T^(s mod h))
//   (tables from gen_tables.py), which is 3-6 orders more accurate than
//   forming A^-1 and A^-T Q A^-1 in FP64.
// * The block-tridiagonal SPD system is solved by block Thomas elimination
//   with h x h Cholesky factors: S_v = D_v - E_{v-1}^T G_{v-1},
//   [G_v | z_v] = S_v^-1 [E_v | rhs_v], back: x_v = z_v - G_v x_{v+1}.
//
// Mapping to CDNA4: a trajectory is owned by a group of LG lanes (LG = 8 for
// N=10, D=3, so 8 trajectories per wave64).  Lane c < h owns column c of
// [E_v | G_v]; lane h + d owns dimension d's right-hand side.  Per vertex every
// lane forms its column with four h x h (or h x N) mat-vecs against Htilde held
// in the scalar cache, the h columns of S_v are exchanged through LDS, every
// lane factors the h x h S_v redundantly in registers (SIMD: redundancy is
// free), and solves its own column.  G_v and z_v stay in LDS for the backward
// sweep, which also recovers coefficients and the cost and streams them to HBM.
// Everything is FP64 (the reference is FP64 throughout).
#include "mtg_internal.h"
#include "mtg.h"
#include "mtg_tables.inc"

#include <float.h>

namespace mtg {

__constant__ double c_a1inv[MTG_A1INV_SIZE] = {MTG_A1INV_VALUES};
__constant__ double c_htilde[MTG_HTILDE_SIZE] = {MTG_HTILDE_VALUES};

// Block of 64 threads = one wave; all LDS traffic is intra-wave.
constexpr int kBlock = 64;
constexpr size_t kMaxLdsPerBlock = 64 * 1024;
constexpr size_t kMaxLdsHard = 160 * 1024;

// s[k] = T^k (k < H) and sc = T^(1-2r): the time-scaling of one segment.
template <int H>
__device__ __forceinline__ void seg_powers(double T, int r, double (&s)[H], double& sc) {
  s[0] = 1.0;
#pragma unroll
  for (int k = 1; k < H; ++k) s[k] = s[k - 1] * T;
  double p = 1.0;
  for (int i = 0; i < 2 * r - 1; ++i) p *= T;
  sc = (r == 0) ? T : 1.0 / p;
}

__device__ __forceinline__ bool time_ok(double T) { return T >= DBL_EPSILON && T <= DBL_MAX; }

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

// Factor the h x h SPD matrix S (lower triangle used) as L L^T; dinv = 1/diag(L).
// Returns false on a non-positive or non-finite pivot.
template <int H>
__device__ __forceinline__ bool chol(const double (&S)[H][H], double (&L)[H][H], double (&dinv)[H]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    double s = S[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
    ok = ok && (s > 0.0) && (s <= DBL_MAX);
    const double l = sqrt(s);
    const double inv = 1.0 / l;
    L[j][j] = l;
    dinv[j] = inv;
#pragma unroll
    for (int i = j + 1; i < H; ++i) {
      double t = S[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
      L[i][j] = t * inv;
    }
  }
  return ok;
}

// x = (L L^T)^-1 b
template <int H>
__device__ __forceinline__ void chol_solve(const double (&L)[H][H], const double (&dinv)[H],
                                           const double (&b)[H], double (&x)[H]) {
  double y[H];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    double t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t -= L[i][k] * y[k];
    y[i] = t * dinv[i];
  }
#pragma unroll
  for (int i = H - 1; i >= 0; --i) {
    double t = y[i];
#pragma unroll
    for (int k = i + 1; k < H; ++k) t -= L[k][i] * x[k];
    x[i] = t * dinv[i];
  }
}

// Per-trajectory LDS slot (doubles): exchange buffer, G_v (K x h x h), z_v (V x D x h).
__host__ __device__ __forceinline__ int slot_doubles(int H, int D, int K, int LG) {
  const int sb = (H * H > LG ? H * H : LG);
  return sb + K * H * H + (K + 1) * D * H;
}

template <int N>
__global__ __launch_bounds__(kBlock) void solve_fused_kernel(SolveArgs a, int lg_log2) {
  constexpr int H = N / 2;
  constexpr unsigned HMASK = (1u << H) - 1u;
  extern __shared__ __attribute__((aligned(16))) double lds[];

  const int LG = 1 << lg_log2;
  const int lane = threadIdx.x;
  const int slot = lane >> lg_log2;
  const int c = lane & (LG - 1);
  const int tpb = kBlock >> lg_log2;
  const int64_t pair = (int64_t)blockIdx.x * tpb + slot;
  const bool valid = pair < a.B;
  const int K = a.K, V = K + 1, D = a.D, r = a.r;
  const bool is_g = c < H;
  const bool is_d = (c >= H) && (c < H + D);
  const int d = is_d ? c - H : 0;
  const int cs = is_g ? c : 0;  // shift amount kept < 32 on non-column lanes
  const int64_t pb = valid ? pair : 0;
  const int64_t tb = pb / a.n_cand;
  const double tscale = a.scales ? a.scales[pb % a.n_cand] : 1.0;

  double* sbuf = lds + (size_t)slot * slot_doubles(H, D, K, LG);
  const int sb = (H * H > LG ? H * H : LG);
  double* gst = sbuf + sb;
  double* zst = gst + K * H * H;

  const double* Ht = c_htilde + (MTG_HTILDE_BASE(N) + r * N * N);
  const double* Ai1 = c_a1inv + MTG_A1INV_OFF(N);
  const double* vals = a.values + tb * (int64_t)V * H * D;
  const uint8_t* msk = a.mask + tb * V;
  const double* tms = a.times + tb * K;

  int st = 0;
  int n_free = 0;

  // ---------------- forward block-Thomas sweep over vertices ----------------
  unsigned raw = msk[0];
  if (raw & ~HMASK) st |= MTG_TRAJ_WARN_DROPPED;
  unsigned m_cur = raw & HMASK;
  raw = msk[1];
  if (raw & ~HMASK) st |= MTG_TRAJ_WARN_DROPPED;
  unsigned m_next = raw & HMASK;
  double xf_cur[H], xf_next[H], gp[H], wz[H];
  load_fixed<H>(vals, 0, D, d, m_cur, xf_cur);
  load_fixed<H>(vals, 1, D, d, m_next, xf_next);
#pragma unroll
  for (int k = 0; k < H; ++k) gp[k] = 0.0, wz[k] = 0.0;
  double T_prev = 0.0, T_next = tms[0] * tscale;
  if (!time_ok(T_next)) st |= MTG_TRAJ_BAD_TIME;

  for (int v = 0; v < V; ++v) {
    const bool has_prev = v > 0, has_next = v < K;
    double a1[H], a2[H], a34[H], m[H], y[H];
    const bool c_free_cur = !((m_cur >> cs) & 1u);
    const bool c_free_next = !((m_next >> cs) & 1u);
#pragma unroll
    for (int k = 0; k < H; ++k) {
      const double ek = (k == c) ? 1.0 : 0.0;
      a1[k] = is_g ? (c_free_cur ? ek : 0.0) : xf_cur[k];
      a2[k] = is_g ? -gp[k] : wz[k];
      a34[k] = is_g ? (c_free_next ? ek : 0.0) : xf_next[k];
      m[k] = 0.0;
      y[k] = 0.0;
    }
    if (has_prev) {
      // H_{v-1} bottom rows: [BL | BR] . [a2 ; a1]  (E_{v-1}^T a2 + D_v^(prev) a1)
      double sp[H], scp;
      seg_powers<H>(T_prev, r, sp, scp);
      double u[N];
#pragma unroll
      for (int k = 0; k < H; ++k) u[k] = sp[k] * a2[k], u[H + k] = sp[k] * a1[k];
#pragma unroll
      for (int i = 0; i < H; ++i) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) acc += Ht[(H + i) * N + j] * u[j];
        m[i] = scp * sp[i] * acc;
      }
    }
    if (has_next) {
      // H_v top rows: TL . a1 (D_v^(next) a1) and TR . a34 (E_v a34)
      double sn[H], scn;
      seg_powers<H>(T_next, r, sn, scn);
      double w1[H], w3[H];
#pragma unroll
      for (int k = 0; k < H; ++k) w1[k] = sn[k] * a1[k], w3[k] = sn[k] * a34[k];
#pragma unroll
      for (int i = 0; i < H; ++i) {
        double acc1 = 0.0, acc3 = 0.0;
#pragma unroll
        for (int j = 0; j < H; ++j) {
          acc1 += Ht[i * N + j] * w1[j];
          acc3 += Ht[i * N + H + j] * w3[j];
        }
        m[i] += scn * sn[i] * acc1;
        y[i] = scn * sn[i] * acc3;
      }
    }
    // Column c of the pinned S_v (G lanes) and the right-hand side.
    double rhs[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const bool fi = !((m_cur >> i) & 1u);
      const double scol = c_free_cur ? (fi ? m[i] : 0.0) : (i == c ? 1.0 : 0.0);
      rhs[i] = is_g ? (fi ? y[i] : 0.0) : (fi ? -(m[i] + y[i]) : 0.0);
      if (is_g) sbuf[c * H + i] = scol;
    }
    __syncthreads();
    double S[H][H];
#pragma unroll
    for (int i = 0; i < H; ++i)
#pragma unroll
      for (int j = 0; j <= i; ++j) S[i][j] = sbuf[j * H + i];
    __syncthreads();
    double L[H][H], dinv[H], x[H];
    if (!chol<H>(S, L, dinv)) st |= MTG_TRAJ_NOT_SPD;
    chol_solve<H>(L, dinv, rhs, x);
    if (is_g && has_next) {
#pragma unroll
      for (int i = 0; i < H; ++i) gst[(v * H + c) * H + i] = x[i], gp[i] = x[i];
    }
    if (is_d) {
#pragma unroll
      for (int i = 0; i < H; ++i) zst[(v * D + d) * H + i] = x[i], wz[i] = xf_cur[i] + x[i];
    }
    n_free += __builtin_popcount(~m_cur & HMASK);
    if (has_next) {
      m_cur = m_next;
#pragma unroll
      for (int k = 0; k < H; ++k) xf_cur[k] = xf_next[k];
      T_prev = T_next;
      if (v + 1 < K) {
        raw = msk[v + 2];
        if (raw & ~HMASK) st |= MTG_TRAJ_WARN_DROPPED;
        m_next = raw & HMASK;
        load_fixed<H>(vals, v + 2, D, d, m_next, xf_next);
        T_next = tms[v + 1] * tscale;
        if (!time_ok(T_next)) st |= MTG_TRAJ_BAD_TIME;
      } else {
        m_next = 0;
#pragma unroll
        for (int k = 0; k < H; ++k) xf_next[k] = 0.0;
        T_next = 0.0;
      }
    }
  }

  // ------------- backward sweep: x_v, coefficients, free values, cost -------------
  double cacc = 0.0;
  if (is_d) {
    double xn[H], xfn[H];
#pragma unroll
    for (int k = 0; k < H; ++k) xn[k] = 0.0, xfn[k] = 0.0;
    int idx = n_free;
    const int64_t fstride = (int64_t)V * H;
    for (int v = K; v >= 0; --v) {
      const unsigned mv = msk[v] & HMASK;
      double x[H], xf[H], xfull[H];
#pragma unroll
      for (int i = 0; i < H; ++i) x[i] = zst[(v * D + d) * H + i];
      if (v < K) {
#pragma unroll
        for (int cc = 0; cc < H; ++cc) {
          const double xc = xn[cc];
#pragma unroll
          for (int i = 0; i < H; ++i) x[i] -= gst[(v * H + cc) * H + i] * xc;
        }
      }
      load_fixed<H>(vals, v, D, d, mv, xf);
#pragma unroll
      for (int i = 0; i < H; ++i) xfull[i] = x[i] + xf[i];
      if (v < K) {
        const double T = tms[v] * tscale;
        double s[H], sc;
        seg_powers<H>(T, r, s, sc);
        double sh[N];
#pragma unroll
        for (int k = 0; k < H; ++k) sh[k] = s[k] * xfull[k], sh[H + k] = s[k] * xfn[k];
        if (a.coeffs) {
          // c = diag(T^-j) A(1)^-1 (S [x_v; x_{v+1}]); A(1)^-1 top-left = diag(1/k!), top-right = 0
          const double tinv = 1.0 / T;
          double out[N];
          double tp = 1.0;
#pragma unroll
          for (int j = 0; j < N; ++j) {
            double acc;
            if (j < H) {
              acc = Ai1[j * N + j] * sh[j];
            } else {
              acc = 0.0;
#pragma unroll
              for (int q = 0; q < N; ++q) acc += Ai1[j * N + q] * sh[q];
            }
            out[j] = acc * tp;
            tp *= tinv;
          }
          if (valid) {
            double2* dst = reinterpret_cast<double2*>(a.coeffs + ((pb * K + v) * D + d) * N);
#pragma unroll
            for (int j = 0; j < N / 2; ++j) dst[j] = make_double2(out[2 * j], out[2 * j + 1]);
          }
        }
        if (a.cost_out) {
          double q = 0.0;
#pragma unroll
          for (int i = 0; i < N; ++i) {
            double row = 0.0;
#pragma unroll
            for (int j = 0; j < N; ++j) row += Ht[i * N + j] * sh[j];
            q += sh[i] * row;
          }
          cacc += sc * q;
        }
      }
      if (a.free_out && valid) {
        double* fo = a.free_out + (pb * D + d) * fstride;
#pragma unroll
        for (int k = H - 1; k >= 0; --k)
          if (!((mv >> k) & 1u)) fo[--idx] = x[k];
      }
#pragma unroll
      for (int k = 0; k < H; ++k) xn[k] = x[k], xfn[k] = xfull[k];
    }
  }
  // cost: sum over dimensions in a fixed order (deterministic)
  if (a.cost_out) {
    __syncthreads();
    if (is_d) sbuf[d] = cacc;
    __syncthreads();
    if (c == H && valid) {
      double tot = 0.0;
      for (int q = 0; q < D; ++q) tot += sbuf[q];
      a.cost_out[pb] = 0.5 * tot;
    }
  }
  if (c == 0 && valid) {
    if (a.status) a.status[pb] = st;
    if (a.n_free_out) a.n_free_out[pb] = n_free;
  }
}

bool solve_geometry(int N, int D, int K, int* lanes_per_traj, size_t* lds_bytes, int* traj_per_block) {
  const int H = N / 2;
  const int need = H + D;
  int lg = 8;
  while (lg < need) lg *= 2;
  if (lg > 64) return false;
  for (;;) {
    const size_t bytes = (size_t)(kBlock / lg) * slot_doubles(H, D, K, lg) * sizeof(double);
    if (bytes <= kMaxLdsPerBlock || (lg == 64 && bytes <= kMaxLdsHard)) {
      *lanes_per_traj = lg;
      *lds_bytes = bytes;
      *traj_per_block = kBlock / lg;
      return true;
    }
    if (lg == 64) return false;
    lg *= 2;
  }
}

template <int N>
static hipError_t launch_fused_n(const SolveArgs& a, hipStream_t stream) {
  int lg, tpb;
  size_t lds;
  if (!solve_geometry(N, a.D, a.K, &lg, &lds, &tpb)) return hipErrorInvalidValue;
  int lg_log2 = 0;
  while ((1 << lg_log2) < lg) ++lg_log2;
  const int64_t blocks = (a.B + tpb - 1) / tpb;
  if (blocks == 0) return hipSuccess;
  if (lds > kMaxLdsPerBlock) {
    hipError_t e = hipFuncSetAttribute((const void*)solve_fused_kernel<N>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(solve_fused_kernel<N>, dim3((unsigned)blocks), dim3(kBlock), lds, stream, a, lg_log2);
  return hipGetLastError();
}

hipError_t launch_solve(int N, const SolveArgs& a, hipStream_t stream) {
  switch (N) {
    case 2: return launch_fused_n<2>(a, stream);
    case 4: return launch_fused_n<4>(a, stream);
    case 6: return launch_fused_n<6>(a, stream);
    case 8: return launch_fused_n<8>(a, stream);
    case 10: return launch_fused_n<10>(a, stream);
    case 12: return launch_fused_n<12>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
