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
#include "mtg_device.h"

#include <stdlib.h>

namespace mtg {

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

  // ---- forward block-Thomas sweep on the symmetrically pinned system (fixed rows AND columns
  // of R replaced by the identity, fixed values moved to the right-hand side):
  //   S_v = D_v - E_{v-1}^T G_{v-1},  [G_v | z_v] = S_v^-1 [E_v | rhs_v],
  //   rhs_v = -(D_v xf_v + E_{v-1}^T (xf_{v-1} + z_{v-1}) + E_v xf_{v+1})   (free rows).
  // Every lane runs the same four mat-vecs against Htilde per vertex with its own inputs:
  //   column lane c:  a1 = e_c (column c of D_v), a2 = -g_{v-1}, a3 = e_c (column c of E_v)
  //   dim lane d:     a1 = xf_v, a2 = xf_{v-1} + z_{v-1}, a3 = xf_{v+1}
  int st = 0, n_free = 0;
  double pmin = DBL_MAX;
  double gp[H], xfc[H], xfn[H];
#pragma unroll
  for (int k = 0; k < H; ++k) gp[k] = 0.0;
  double sp[H], scp = 0.0, sn[H], scn = 0.0;
#pragma unroll
  for (int k = 0; k < H; ++k) sp[k] = 0.0;
  {
    const double T0 = tms[0] * tscale;
    st |= time_bits(T0);
    seg_powers<H, R>(T0, sn, scn);
  }
  unsigned raw = msk[0];
  if (raw & ~HMASK) st |= MTG_TRAJ_WARN_DROPPED;
  unsigned m_cur = raw & HMASK;
  raw = msk[1];
  if (raw & ~HMASK) st |= MTG_TRAJ_WARN_DROPPED;
  unsigned m_next = raw & HMASK;
  unsigned m_prev = 0;
  double xfp0 = 0.0;  // fixed position of vertex v-1 (dim lanes)
  load_fixed<H>(vals, 0, D, d, m_cur, xfc);
  load_fixed<H>(vals, 1, D, d, m_next, xfn);
  for (int v = 0; v < V; ++v) {
    const bool has_prev = v > 0, has_next = v < K;
    cdouble* Hs = launder(Ht);
    const bool c_free = !((m_cur >> cs) & 1u);
    const bool c_free_next = !((m_next >> cs) & 1u);
    double a1[H], a2[H], a3[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      const double ek = (k == c) ? 1.0 : 0.0;
      a1[k] = is_g ? (c_free ? ek : 0.0) : xfc[k];
      a2[k] = gp[k];  // column lanes keep -g_{v-1}, dim lanes xf_{v-1} + z_{v-1}
      a3[k] = is_g ? (c_free_next ? ek : 0.0) : xfn[k];
    }
    // Translation invariance (r >= 1: H_i [1 0..0 1 0..0]^T = 0): for a segment whose two end
    // positions are both fixed, the fixed-value products use positions relative to the segment
    // start.  Exact in real arithmetic; in FP64 it removes the cancellation of
    // H^TL p_v + H^TR p_{v+1} on short segments (up to 500x more accurate, DESIGN.md "Numerics").
    double a1b0 = a1[0];
    if (R >= 1 && is_d) {
      const bool pos_c = m_cur & 1u, pos_p = m_prev & 1u, pos_n = m_next & 1u;
      if (has_prev && pos_p && pos_c) {  // segment v-1: positions relative to p_{v-1}
        a1b0 = xfc[0] - xfp0;
        a2[0] = 0.0;
      }
      if (has_next && pos_c && pos_n) {  // segment v: positions relative to p_v
        a3[0] = xfn[0] - xfc[0];
        a1[0] = 0.0;
      }
    }
    double m[H], y[H];
#pragma unroll
    for (int i = 0; i < H; ++i) m[i] = 0.0, y[i] = 0.0;
    if (has_prev) {  // bottom rows of H_{v-1}: [BL | BR] [a2; a1]
      double u[N];
#pragma unroll
      for (int k = 0; k < H; ++k) u[k] = sp[k] * a2[k], u[H + k] = sp[k] * a1[k];
      u[H] = a1b0;  // sp[0] == 1
#pragma unroll
      for (int i = 0; i < H; ++i) {
        double t = 0.0;
#pragma unroll
        for (int j = 0; j < N; ++j) t += Hs[(H + i) * N + j] * u[j];
        m[i] = scp * sp[i] * t;
      }
    }
    if (has_next) {  // top rows of H_v: TL a1 and TR a3
      double w1[H], w3[H];
#pragma unroll
      for (int k = 0; k < H; ++k) w1[k] = sn[k] * a1[k], w3[k] = sn[k] * a3[k];
#pragma unroll
      for (int i = 0; i < H; ++i) {
        double t1 = 0.0, t3 = 0.0;
#pragma unroll
        for (int j = 0; j < H; ++j) {
          t1 += Hs[i * N + j] * w1[j];
          t3 += Hs[i * N + H + j] * w3[j];
        }
        const double f = scn * sn[i];
        m[i] += f * t1;
        y[i] = f * t3;
      }
    }
    double rhs[H];
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const bool fi = !((m_cur >> i) & 1u);
      double sv = c_free ? (fi ? m[i] : 0.0) : (i == c ? 1.0 : 0.0);
      double rg = fi ? y[i] : 0.0;
      double rd = fi ? -(m[i] + y[i]) : 0.0;
      asm volatile("" : "+v"(sv), "+v"(rg), "+v"(rd));  // all computed: branch-free selects
      xs[c * H + i] = sv;  // only columns c < H are read
      rhs[i] = is_g ? rg : rd;
    }
    __syncthreads();
    double S[H][H];
#pragma unroll
    for (int i = 0; i < H; ++i)
#pragma unroll
      for (int j = 0; j <= i; ++j) S[i][j] = xs[j * H + i];
    __syncthreads();
    double dinv[H], x[H];
    const double pv = ldlt<H>(S, dinv);
    pmin = (pv < pmin || pv != pv) ? pv : pmin;  // a NaN pivot sticks (NOT_SPD)
    ldlt_solve<H>(S, dinv, rhs, x);
    if (is_g && has_next) {
#pragma unroll
      for (int i = 0; i < H; ++i) gst[(v * H + c) * H + i] = x[i];
    }
    if (is_d) {
#pragma unroll
      for (int i = 0; i < H; ++i) zst[(v * D + d) * H + i] = x[i];
    }
#pragma unroll
    for (int i = 0; i < H; ++i) gp[i] = is_g ? -x[i] : xfc[i] + x[i];
    n_free += __builtin_popcount(~m_cur & HMASK);
    if (has_next) {
      xfp0 = xfc[0];
      m_prev = m_cur;
#pragma unroll
      for (int k = 0; k < H; ++k) sp[k] = sn[k], xfc[k] = xfn[k];
      scp = scn;
      m_cur = m_next;
      if (v + 1 < K) {
        const double Tn = tms[v + 1] * tscale;
        st |= time_bits(Tn);
        seg_powers<H, R>(Tn, sn, scn);
        raw = msk[v + 2];
        if (raw & ~HMASK) st |= MTG_TRAJ_WARN_DROPPED;
        m_next = raw & HMASK;
        load_fixed<H>(vals, v + 2, D, d, m_next, xfn);
      } else {
        m_next = 0;
#pragma unroll
        for (int k = 0; k < H; ++k) xfn[k] = 0.0;
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
  // Items (segment i, dimension dd) go in rounds of LG, item it = base + c.  A round's coefficient
  // rows are consecutive in HBM ([K][D][N] per trajectory): when the G store (dead after the
  // backward sweep) can hold them they are staged there and stored as one contiguous run per
  // trajectory, 16 B per lane at consecutive addresses (per-lane 16-B pieces at an N-double
  // stride kept the store unit busy for most of the epilogue; see mtg_solve_reg.inc).
  const bool stage = K * H * H >= LG * N && !(slot_doubles(H, D, K, LG) & 1);  // room, 16-B aligned
  for (int base = 0; base < K * D; base += LG) {
    const int it = base + c;
    const bool have = it < K * D;
    const int i = have ? it / D : 0, dd = have ? it - i * D : 0;
    cdouble* Hl = launder(c_htilde + MTG_HTILDE_OFF(N, R));
    cdouble* Ai1 = launder(c_a1inv + MTG_A1INV_OFF(N));
    const double T = tms[i] * tscale;
    double s[H], sc;
    seg_powers<H, R>(T, s, sc);
    double x0[H], x1[H];
    load_fixed<H>(vals, i, D, dd, msk[i], x0);
    load_fixed<H>(vals, i + 1, D, dd, msk[i + 1], x1);
    double sh[N];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      sh[k] = s[k] * (x0[k] + zst[(i * D + dd) * H + k]);
      sh[H + k] = s[k] * (x1[k] + zst[((i + 1) * D + dd) * H + k]);
    }
    // the polynomial of [x_i - p 1; x_{i+1} - p 1] is p(t) - p: recover it relative to the start
    // position p (only c_0 changes), which avoids cancelling p_i against p_{i+1} in c_j, j >= h
    const double p0 = sh[0];
    sh[0] = 0.0;
    sh[H] -= p0;
    if (a.coeffs) {
      const double tinv = rcp(T);
      double out[N];
      double tp = 1.0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        double acc;
        if (j < H) {  // A(1)^-1 top-left = diag(1/j!), top-right = 0
          acc = (j == 0) ? p0 : Ai1[j * N + j] * sh[j];
        } else {
          acc = 0.0;
#pragma unroll
          for (int q = 0; q < N; ++q) acc += Ai1[j * N + q] * sh[q];
        }
        out[j] = acc * tp;
        tp *= tinv;
      }
      if (stage) {
        double2* o2 = reinterpret_cast<double2*>(gst + c * N);
#pragma unroll
        for (int j = 0; j < N / 2; ++j) o2[j] = make_double2(out[2 * j], out[2 * j + 1]);
        __syncthreads();  // (one wave per block: orders the LDS staging)
        const int nrun = (K * D - base < LG ? K * D - base : LG) * (N / 2);  // double2s this round
        if (valid) {
          double2* dst = reinterpret_cast<double2*>(a.coeffs + (pb * (K * D) + base) * N);
          const double2* src = reinterpret_cast<const double2*>(gst);
          for (int e = c; e < nrun; e += LG) store_stream(dst + e, src[e]);
        }
        __syncthreads();
      } else if (valid && have) {
        double2* dst = reinterpret_cast<double2*>(a.coeffs + ((pb * K + i) * D + dd) * N);
#pragma unroll
        for (int j = 0; j < N / 2; ++j) store_stream(dst + j, make_double2(out[2 * j], out[2 * j + 1]));
      }
    }
    if (a.cost_out && have) {  // 0.5 c^T Q c = 0.5 sc sh^T Htilde sh  (translation-invariant for r >= 1)
      if (R == 0) sh[0] = p0, sh[H] += p0;
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
  static const size_t lds_pad = [] {  // occupancy experiments only (DESIGN.md "Occupancy")
    const char* p = getenv("MTG_DEBUG_LDS_PAD");
    return p ? (size_t)atoi(p) : (size_t)0;
  }();
  lds += lds_pad;
  if (lds > kMaxLdsPerBlock) {
    hipError_t e = hipFuncSetAttribute((const void*)solve_fused_kernel<N, R>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  launch_kernel((solve_fused_kernel<N, R>), dim3((unsigned)blocks), dim3(kBlock), lds, stream, a, lg_log2);
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

int solve_kernel(int N, int D, int K, unsigned flags, int r, int64_t B) {
  int lg;
  size_t lds;
  if (flags & MTG_FLAG_GENERAL_KERNEL) return MTG_KERNEL_GENERAL;
  if ((flags & MTG_FLAG_LANE_KERNEL) && lane_geometry(N, D, K, &lds)) return MTG_KERNEL_LANE;
  if ((flags & MTG_FLAG_IP_KERNEL) && r >= 0 && ip_geometry(N, D, K, r)) return MTG_KERNEL_IP;
  // the dimension-lane kernel: asked for, or by default for large batches (at
  // B = 125000 ~15% faster than the column kernel, at 1e4 within the box-to-box spread)
  const bool dl_default = B >= MTG_DL_MIN_BATCH && !(flags & MTG_FLAG_COLUMN_KERNEL);
  if (((flags & MTG_FLAG_DL_KERNEL) || dl_default) && r >= 0 && dl_geometry(N, D, K, r)) return MTG_KERNEL_DL;
  if (reg_geometry(N, D, K, &lg, &lds)) return MTG_KERNEL_COLUMN;
  return MTG_KERNEL_GENERAL;
}

hipError_t launch_solve(int N, const SolveArgs& a, hipStream_t stream, unsigned flags) {
  switch (solve_kernel(N, a.D, a.K, flags, a.r, a.B)) {
    case MTG_KERNEL_LANE: return launch_solve_lane(N, a, stream);
    case MTG_KERNEL_IP: return launch_solve_ip(N, a, stream);
    case MTG_KERNEL_DL: return launch_solve_dl(N, a, stream);
    case MTG_KERNEL_COLUMN: return launch_solve_reg(N, a, stream);
    default: break;
  }
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
