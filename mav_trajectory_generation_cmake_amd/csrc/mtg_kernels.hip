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

// In-place LU without pivoting of the h x h pivot block (unit-lower L below the diagonal,
// U on and above it); dinv = 1/diag(U).  The block's fixed rows are identity rows (pivot 1)
// and its free-free part is the SPD Schur complement of R_pp, so no pivoting is needed.
// Returns the smallest pivot (<= 0 or non-finite: R_pp not SPD; the reference never checks,
// lin_impl:355-368).
template <int H>
__device__ __forceinline__ double lu_inplace(double (&S)[H][H], double (&dinv)[H]) {
  double pmin = DBL_MAX;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const double piv = S[k][k];
    pmin = fmin(pmin, piv);
    const double inv = rcp(piv);
    dinv[k] = inv;
#pragma unroll
    for (int i = k + 1; i < H; ++i) {
      const double l = S[i][k] * inv;
      S[i][k] = l;
#pragma unroll
      for (int j = k + 1; j < H; ++j) S[i][j] -= l * S[k][j];
    }
  }
  return pmin;
}

template <int H>
__device__ __forceinline__ void lu_solve(const double (&S)[H][H], const double (&dinv)[H],
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
    double t = y[i];
#pragma unroll
    for (int k = i + 1; k < H; ++k) t -= S[i][k] * x[k];
    x[i] = t * dinv[i];
  }
}

// Per-trajectory LDS slot (doubles): exchange buffer (LG x h), G_v (K x h x h), Z_v (V x D x h:
// z_v after the forward sweep, the solution x_v after the backward sweep).
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

template <int N, int R>
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
  const int K = a.K, V = K + 1, D = a.D;
  const bool is_g = c < H;
  const bool is_d = (c >= H) && (c < H + D);
  const int d = is_d ? c - H : 0;
  const int cs = is_g ? c : 0;
  const int64_t pb = valid ? pair : 0;
  const int64_t tb = pb / a.n_cand;
  const double tscale = a.scales ? a.scales[pb % a.n_cand] : 1.0;

  double* xs = lds + (size_t)slot * slot_doubles(H, D, K, LG);
  double* gst = xs + LG * H;
  double* zst = gst + K * H * H;

  const double* Ht = c_htilde + MTG_HTILDE_OFF(N, R);
  const double* vals = a.values + tb * (int64_t)V * H * D;
  const uint8_t* msk = a.mask + tb * V;
  const double* tms = a.times + tb * K;

  // Htilde columns this lane needs as a column owner (lane-varying index: loaded once).
  double hTL[H], hBR[H], hTR[H];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    hTL[i] = Ht[i * N + cs];
    hBR[i] = Ht[(H + i) * N + H + cs];
    hTR[i] = Ht[i * N + H + cs];
  }

  // ---- forward block-Thomas sweep on the row-pinned system:
  //   S_v = D_v - C_v G_{v-1},  [G_v | z_v] = S_v^-1 [E_v | b_v - C_v z_{v-1}]
  // where C_v / E_v are the lower / upper coupling blocks (H_{v-1} bottom-left, H_v top-right)
  // and fixed rows of S_v, C_v, E_v are replaced by identity / zero rows with the fixed value
  // in b_v.  Lane c < H owns column c of [E_v | G_v], lane H + d the right-hand side of dim d.
  int st = 0, n_free = 0;
  double pmin = DBL_MAX;
  double gprev[H];
#pragma unroll
  for (int k = 0; k < H; ++k) gprev[k] = 0.0;
  double sp[H], scp = 0.0, sn[H], scn = 0.0;
#pragma unroll
  for (int k = 0; k < H; ++k) sp[k] = 0.0;
  {
    const double T0 = tms[0] * tscale;
    if (!time_ok(T0)) st |= MTG_TRAJ_BAD_TIME;
    seg_powers<H, R>(T0, sn, scn);
  }
  unsigned raw = msk[0];
  for (int v = 0; v < V; ++v) {
    const bool has_prev = v > 0, has_next = v < K;
    if (raw & ~HMASK) st |= MTG_TRAJ_WARN_DROPPED;
    const unsigned m_cur = raw & HMASK;
    if (has_next) raw = msk[v + 1];
    // w = C_v gprev  (bottom-left block of H_{v-1}; rows masked below)
    double w[H];
#pragma unroll
    for (int i = 0; i < H; ++i) w[i] = 0.0;
    if (has_prev) {
      double u[H];
#pragma unroll
      for (int k = 0; k < H; ++k) u[k] = sp[k] * gprev[k];
#pragma unroll
      for (int i = 0; i < H; ++i) {
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < H; ++j) t += Ht[(H + i) * N + j] * u[j];
        w[i] = scp * sp[i] * t;
      }
    }
    double val[H];
    {
      const double* p = vals + ((size_t)v * H) * D + d;
#pragma unroll
      for (int k = 0; k < H; ++k) val[k] = p[k * D];
    }
    const double fp = has_prev ? scp * sp[cs] : 0.0;   // column-c factors of the two segments
    const double fnx = has_next ? scn * sn[cs] : 0.0;
    double u[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const bool fi = !((m_cur >> i) & 1u);
      const double dcol = fp * sp[i] * hBR[i] + fnx * sn[i] * hTL[i];  // column c of D_v
      const double ecol = fnx * sn[i] * hTR[i];                        // column c of E_v
      xs[c * H + i] = fi ? dcol - w[i] : (i == c ? 1.0 : 0.0);         // only c < H is read
      double ug = fi ? ecol : 0.0;
      double ud = fi ? -w[i] : val[i];
      asm volatile("" : "+v"(ug), "+v"(ud));  // both computed: branch-free selects
      u[i] = is_g ? ug : ud;
    }
    __syncthreads();
    double S[H][H];
#pragma unroll
    for (int i = 0; i < H; ++i)
#pragma unroll
      for (int j = 0; j < H; ++j) S[i][j] = xs[j * H + i];
    __syncthreads();
    double dinv[H], x[H];
    pmin = fmin(pmin, lu_inplace<H>(S, dinv));
    lu_solve<H>(S, dinv, u, x);
    if (is_g && has_next) {
#pragma unroll
      for (int i = 0; i < H; ++i) gst[(v * H + c) * H + i] = x[i];
    }
    if (is_d) {
#pragma unroll
      for (int i = 0; i < H; ++i) zst[(v * D + d) * H + i] = x[i];
    }
#pragma unroll
    for (int i = 0; i < H; ++i) gprev[i] = x[i];
    n_free += __builtin_popcount(~m_cur & HMASK);
    if (has_next) {
#pragma unroll
      for (int k = 0; k < H; ++k) sp[k] = sn[k];
      scp = scn;
      if (v + 1 < K) {
        const double Tn = tms[v + 1] * tscale;
        if (!time_ok(Tn)) st |= MTG_TRAJ_BAD_TIME;
        seg_powers<H, R>(Tn, sn, scn);
      }
    }
  }
  if (!(pmin > 0.0 && pmin <= DBL_MAX)) st |= MTG_TRAJ_NOT_SPD;
  __syncthreads();

  // ---- backward substitution (dimension lanes): x_v = z_v - G_v x_{v+1}, kept in Z
  if (is_d) {
    double xn[H];
#pragma unroll
    for (int k = 0; k < H; ++k) xn[k] = zst[(K * D + d) * H + k];
    for (int v = K - 1; v >= 0; --v) {
      double x[H];
#pragma unroll
      for (int i = 0; i < H; ++i) x[i] = zst[(v * D + d) * H + i];
#pragma unroll
      for (int cc = 0; cc < H; ++cc) {
        const double xc = xn[cc];
#pragma unroll
        for (int i = 0; i < H; ++i) x[i] -= gst[(v * H + cc) * H + i] * xc;
      }
#pragma unroll
      for (int i = 0; i < H; ++i) zst[(v * D + d) * H + i] = x[i], xn[i] = x[i];
    }
  }
  __syncthreads();

  // ---- epilogue: coefficients c = diag(T^-j) A(1)^-1 S(T) [x_i; x_{i+1}] and the cost, items (i, d)
  double cacc = 0.0;
  for (int it = c; it < K * D; it += LG) {
    const int i = it / D, dd = it - i * D;
    cdouble* Hl = launder(c_htilde + MTG_HTILDE_OFF(N, R));
    cdouble* Ai1 = launder(c_a1inv + MTG_A1INV_OFF(N));
    const double T = tms[i] * tscale;
    double s[H], sc;
    seg_powers<H, R>(T, s, sc);
    double sh[N];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      sh[k] = s[k] * zst[(i * D + dd) * H + k];
      sh[H + k] = s[k] * zst[((i + 1) * D + dd) * H + k];
    }
    if (a.coeffs) {
      const double tinv = rcp(T);
      double out[N];
      double tp = 1.0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        double acc;
        if (j < H) {  // A(1)^-1 top-left = diag(1/j!), top-right = 0
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
        double2* dst = reinterpret_cast<double2*>(a.coeffs + ((pb * K + i) * D + dd) * N);
#pragma unroll
        for (int j = 0; j < N / 2; ++j) dst[j] = make_double2(out[2 * j], out[2 * j + 1]);
      }
    }
    if (a.cost_out) {  // 0.5 c^T Q c = 0.5 sc sh^T Htilde sh
      double q = 0.0;
#pragma unroll
      for (int p = 0; p < N; ++p) {
        double row = 0.5 * Hl[p * N + p] * sh[p];
#pragma unroll
        for (int t = p + 1; t < N; ++t) row += Hl[p * N + t] * sh[t];
        q += sh[p] * row;
      }
      cacc += sc * q;
    }
  }
  // free derivatives in the reference order (sorted by vertex, then derivative)
  if (a.free_out && valid && is_d) {
    double* fo = a.free_out + (pb * D + d) * ((int64_t)V * H);
    int idx = 0;
    for (int v = 0; v < V; ++v) {
      const unsigned mv = msk[v] & HMASK;
#pragma unroll
      for (int k = 0; k < H; ++k)
        if (!((mv >> k) & 1u)) fo[idx++] = zst[(v * D + d) * H + k];
    }
  }
  if (a.cost_out) {  // fixed-order reduction over the group's lanes (deterministic)
    __syncthreads();
    xs[c] = cacc;
    __syncthreads();
    if (c == 0 && valid) {
      double tot = 0.0;
      for (int q = 0; q < LG; ++q) tot += xs[q];
      a.cost_out[pb] = tot;
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

template <int N, int R>
static hipError_t launch_fused_nr(const SolveArgs& a, hipStream_t stream) {
  int lg, tpb;
  size_t lds;
  if (!solve_geometry(N, a.D, a.K, &lg, &lds, &tpb)) return hipErrorInvalidValue;
  int lg_log2 = 0;
  while ((1 << lg_log2) < lg) ++lg_log2;
  const int64_t blocks = (a.B + tpb - 1) / tpb;
  if (blocks == 0) return hipSuccess;
  if (lds > kMaxLdsPerBlock) {
    hipError_t e = hipFuncSetAttribute((const void*)solve_fused_kernel<N, R>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((solve_fused_kernel<N, R>), dim3((unsigned)blocks), dim3(kBlock), lds, stream, a, lg_log2);
  return hipGetLastError();
}

template <int N>
static hipError_t launch_fused_n(const SolveArgs& a, hipStream_t stream) {
  switch (a.r) {
    case 0: return launch_fused_nr<N, 0>(a, stream);
    case 1: if constexpr (N / 2 > 1) return launch_fused_nr<N, 1>(a, stream); break;
    case 2: if constexpr (N / 2 > 2) return launch_fused_nr<N, 2>(a, stream); break;
    case 3: if constexpr (N / 2 > 3) return launch_fused_nr<N, 3>(a, stream); break;
    case 4: if constexpr (N / 2 > 4) return launch_fused_nr<N, 4>(a, stream); break;
    case 5: if constexpr (N / 2 > 5) return launch_fused_nr<N, 5>(a, stream); break;
    default: break;
  }
  return hipErrorInvalidValue;
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
