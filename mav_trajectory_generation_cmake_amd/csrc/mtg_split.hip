// mtg_split.hip -- the two-kernel solve path (MTG_FLAG_SPLIT_KERNELS).
//
// The same minimiser as the fused kernels, cut at the boundary the reference itself has between
// building R (constructR, lin_impl:298-326) and solving it (solveLinear's SparseQR, :329-369), so
// each half can be profiled on its own:
//   assemble_kernel        one thread per (trajectory, vertex): the pinned block-tridiagonal system
//                          D_v (h x h, symmetric), E_v (coupling v -> v+1) and the right-hand side
//                          b_v = -(R x_f)_v (h x D) from the exact-rational Htilde table and the
//                          segment times; fixed positions enter translation-relative (DESIGN.md
//                          "Numerics").  Written to an HBM workspace.
//   block_cholesky_kernel  one thread per trajectory: block LDL^T Thomas sweep over the workspace
//                          (G_v = S_v^-1 E_v and z_v stored in place of E_v and b_v), back
//                          substitution, then coefficient recovery, cost, free values and status.
// Workspace layout: ws[(v * NE + e) * B + b], e over {D_v lower triangle (h(h+1)/2), E_v (h*h,
// row-major), b_v (h*D, [i][d])}: the trajectory index is fastest, so every access of both kernels
// is a coalesced 8-byte-per-lane stream.
#include "mtg_device.h"

namespace mtg {

namespace split {

__host__ __device__ constexpr int tri(int h) { return h * (h + 1) / 2; }
__host__ __device__ inline int ws_elems(int H, int D) { return tri(H) + H * H + H * D; }

// Fixed values of vertex v, dimension d (0 on free derivatives; read only where fixed).
template <int H>
__device__ __forceinline__ void fixed_vals(const double* vals, int v, int D, int d, unsigned m, double (&x)[H]) {
  const double* p = vals + ((size_t)v * H) * D + d;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const double t = p[k * D];
    x[k] = ((m >> k) & 1u) ? t : 0.0;
  }
}

template <int N, int R>
__global__ __launch_bounds__(256) void assemble_kernel(SolveArgs a, double* ws) {
  constexpr int H = N / 2;
  constexpr unsigned HM = (1u << H) - 1u;
  const int K = a.K, V = K + 1, D = a.D;
  const int64_t B = a.B;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * V) return;
  const int v = (int)(gid / B);  // vertex-major over the grid: consecutive threads, consecutive b
  const int64_t b = gid - (int64_t)v * B;
  const int64_t tb = b / a.n_cand;
  const double tscale = a.scales ? a.scales[b % a.n_cand] : 1.0;
  const double* vals = a.values + tb * (int64_t)V * H * D;
  const uint8_t* msk = a.mask + tb * V;
  const double* tms = a.times + tb * K;
  const int NE = ws_elems(H, D);
  double* w = ws + ((int64_t)v * NE) * B + b;  // element e at w[e * B]

  const bool has_prev = v > 0, has_next = v < K;
  const unsigned mp = has_prev ? (msk[v - 1] & HM) : 0u, mc = msk[v] & HM, mn = has_next ? (msk[v + 1] & HM) : 0u;
  double sp[H], sn[H], scp = 0.0, scn = 0.0;
#pragma unroll
  for (int k = 0; k < H; ++k) sp[k] = 0.0, sn[k] = 0.0;
  if (has_prev) seg_powers<H, R>(tms[v - 1] * tscale, sp, scp);
  if (has_next) seg_powers<H, R>(tms[v] * tscale, sn, scn);
  cdouble* Ht = (cdouble*)(c_htilde + MTG_HTILDE_OFF(N, R));

  // D_v = BR_{v-1} + TL_v on free rows/columns, identity on fixed ones (lower triangle)
  int e = 0;
#pragma unroll
  for (int i = 0; i < H; ++i) {
#pragma unroll
    for (int j = 0; j <= i; ++j, ++e) {
      double s = 0.0;
      if (has_prev) s += scp * sp[i] * Ht[(H + i) * N + H + j] * sp[j];
      if (has_next) s += scn * sn[i] * Ht[i * N + j] * sn[j];
      const bool fi = (mc >> i) & 1u, fj = (mc >> j) & 1u;
      w[(int64_t)e * B] = (fi || fj) ? (i == j ? 1.0 : 0.0) : s;
    }
  }
  // E_v = TR_v on (free at v) x (free at v+1), zero elsewhere
#pragma unroll
  for (int i = 0; i < H; ++i) {
#pragma unroll
    for (int j = 0; j < H; ++j, ++e) {
      double s = 0.0;
      if (has_next && !((mc >> i) & 1u) && !((mn >> j) & 1u)) s = scn * sn[i] * Ht[i * N + H + j] * sn[j];
      w[(int64_t)e * B] = s;
    }
  }
  // b_v = -(BL_{v-1} x_f,v-1 + (BR_{v-1} + TL_v) x_f,v + TR_v x_f,v+1) on free rows
  for (int d = 0; d < D; ++d) {
    double xp[H], xc[H], xn[H];
    fixed_vals<H>(vals, v, D, d, mc, xc);
    if (has_prev) fixed_vals<H>(vals, v - 1, D, d, mp, xp);
    else
#pragma unroll
      for (int k = 0; k < H; ++k) xp[k] = 0.0;
    if (has_next) fixed_vals<H>(vals, v + 1, D, d, mn, xn);
    else
#pragma unroll
      for (int k = 0; k < H; ++k) xn[k] = 0.0;
    double xcb[H], xct[H];
#pragma unroll
    for (int k = 0; k < H; ++k) xcb[k] = xc[k], xct[k] = xc[k];
    if (R >= 1) {  // translation-relative positions on segments whose two end positions are fixed
      if (has_prev && (mp & mc & 1u)) xcb[0] = xc[0] - xp[0], xp[0] = 0.0;
      if (has_next && (mc & mn & 1u)) xn[0] = xn[0] - xc[0], xct[0] = 0.0;
    }
#pragma unroll
    for (int i = 0; i < H; ++i) {
      double bot = 0.0, top = 0.0;
      if (has_prev) {
#pragma unroll
        for (int j = 0; j < H; ++j)
          bot += Ht[(H + i) * N + j] * (sp[j] * xp[j]) + Ht[(H + i) * N + H + j] * (sp[j] * xcb[j]);
      }
      if (has_next) {
#pragma unroll
        for (int j = 0; j < H; ++j)
          top += Ht[i * N + j] * (sn[j] * xct[j]) + Ht[i * N + H + j] * (sn[j] * xn[j]);
      }
      const double r = -(scp * sp[i] * bot + scn * sn[i] * top);
      w[(int64_t)(e + i * D + d) * B] = ((mc >> i) & 1u) ? 0.0 : r;
    }
  }
}

template <int N, int R>
__global__ __launch_bounds__(128) void block_cholesky_kernel(SolveArgs a, double* ws) {
  constexpr int H = N / 2;
  constexpr unsigned HM = (1u << H) - 1u;
  constexpr int TR = tri(H);
  const int K = a.K, V = K + 1, D = a.D;
  const int64_t B = a.B;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t tb = b / a.n_cand;
  const double tscale = a.scales ? a.scales[b % a.n_cand] : 1.0;
  const double* vals = a.values + tb * (int64_t)V * H * D;
  const uint8_t* msk = a.mask + tb * V;
  const double* tms = a.times + tb * K;
  const int NE = ws_elems(H, D);
  auto W = [&](int v, int e) -> double& { return ws[((int64_t)v * NE + e) * B + b]; };
  const int EO = TR, BO = TR + H * H;  // offsets of E_v and b_v within a vertex

  int st = 0, n_free = 0;
  double pmin = DBL_MAX;
  for (int v = 0; v < V; ++v) {
    const unsigned raw = msk[v];
    if (raw & ~HM) st |= MTG_TRAJ_WARN_DROPPED;
    n_free += __builtin_popcount(~raw & HM);
    if (v < K) st |= time_bits(tms[v] * tscale);
  }

  // forward: S_v = D_v - E_{v-1}^T G_{v-1}, rhs_v = b_v - E_{v-1}^T z_{v-1}; factor; G_v, z_v
  double Ep[H][H], Gp[H][H];  // E_{v-1}, G_{v-1}
  for (int v = 0; v < V; ++v) {
    double S[H][H];
    {
      int e = 0;
#pragma unroll
      for (int i = 0; i < H; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j, ++e) S[i][j] = W(v, e);
    }
    if (v > 0) {
#pragma unroll
      for (int i = 0; i < H; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
          double t = 0.0;
#pragma unroll
          for (int k = 0; k < H; ++k) t += Ep[k][i] * Gp[k][j];
          S[i][j] -= t;
        }
    }
    double dinv[H];
    const double pv = ldlt<H>(S, dinv);
    pmin = (pv < pmin || pv != pv) ? pv : pmin;  // a NaN pivot sticks (NOT_SPD)
    for (int d = 0; d < D; ++d) {  // z_v
      double r[H], z[H];
#pragma unroll
      for (int i = 0; i < H; ++i) r[i] = W(v, BO + i * D + d);
      if (v > 0) {
#pragma unroll
        for (int i = 0; i < H; ++i) {
          double t = 0.0;
#pragma unroll
          for (int k = 0; k < H; ++k) t += Ep[k][i] * W(v - 1, BO + k * D + d);
          r[i] -= t;
        }
      }
      ldlt_solve<H>(S, dinv, r, z);
#pragma unroll
      for (int i = 0; i < H; ++i) W(v, BO + i * D + d) = z[i];
    }
    if (v < K) {  // G_v = S_v^-1 E_v, stored over E_v
#pragma unroll
      for (int i = 0; i < H; ++i)
#pragma unroll
        for (int j = 0; j < H; ++j) Ep[i][j] = W(v, EO + i * H + j);
#pragma unroll
      for (int j = 0; j < H; ++j) {
        double col[H], g[H];
#pragma unroll
        for (int i = 0; i < H; ++i) col[i] = Ep[i][j];
        ldlt_solve<H>(S, dinv, col, g);
#pragma unroll
        for (int i = 0; i < H; ++i) Gp[i][j] = g[i], W(v, EO + i * H + j) = g[i];
      }
    }
  }
  if (!(pmin > 0.0 && pmin <= DBL_MAX)) st |= MTG_TRAJ_NOT_SPD;

  // backward: x_v = z_v - G_v x_{v+1}, stored over z_v (pinned: the free part, 0 on fixed slots)
  for (int d = 0; d < D; ++d) {
    double xn[H];
#pragma unroll
    for (int i = 0; i < H; ++i) xn[i] = W(K, BO + i * D + d);
    for (int v = K - 1; v >= 0; --v) {
      double x[H];
#pragma unroll
      for (int i = 0; i < H; ++i) {
        double t = W(v, BO + i * D + d);
#pragma unroll
        for (int j = 0; j < H; ++j) t -= W(v, EO + i * H + j) * xn[j];
        x[i] = t;
      }
#pragma unroll
      for (int i = 0; i < H; ++i) W(v, BO + i * D + d) = x[i], xn[i] = x[i];
    }
  }

  // recovery: c = diag(T^-j) A(1)^-1 S(T) [x_i; x_{i+1}] with x = x_f + x_p, translated by p = x_i[0]
  cdouble* Ai1 = (cdouble*)(c_a1inv + MTG_A1INV_OFF(N));
  cdouble* Hl = (cdouble*)(c_htilde + MTG_HTILDE_OFF(N, R));
  double cost = 0.0;
  for (int i = 0; i < K; ++i) {
    const double T = tms[i] * tscale;
    double s[H], sc;
    seg_powers<H, R>(T, s, sc);
    const double tinv = rcp(T);
    const unsigned m0 = msk[i] & HM, m1 = msk[i + 1] & HM;
    for (int d = 0; d < D; ++d) {
      double x0[H], x1[H], sh[N];
      fixed_vals<H>(vals, i, D, d, m0, x0);
      fixed_vals<H>(vals, i + 1, D, d, m1, x1);
#pragma unroll
      for (int k = 0; k < H; ++k) {
        sh[k] = s[k] * (x0[k] + W(i, BO + k * D + d));
        sh[H + k] = s[k] * (x1[k] + W(i + 1, BO + k * D + d));
      }
      const double p0 = sh[0];
      sh[0] = 0.0;
      sh[H] -= p0;
      if (a.coeffs) {
        double* out = a.coeffs + ((b * K + i) * D + d) * N;
        double tp = 1.0;
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
      if (a.cost_out) {
        if (R == 0) sh[0] = p0, sh[H] += p0;
        double q = 0.0;
#pragma unroll
        for (int p = 0; p < N; ++p) {
          double row = 0.5 * Hl[p * N + p] * sh[p];
#pragma unroll
          for (int t = p + 1; t < N; ++t) row += Hl[p * N + t] * sh[t];
          q += sh[p] * row;
        }
        cost += sc * q;
      }
    }
  }
  if (a.free_out) {
    for (int d = 0; d < D; ++d) {
      double* fo = a.free_out + (b * D + d) * ((int64_t)V * H);
      int idx = 0;
      for (int v = 0; v < V; ++v) {
        const unsigned mv = msk[v] & HM;
#pragma unroll
        for (int k = 0; k < H; ++k)
          if (!((mv >> k) & 1u)) fo[idx++] = W(v, BO + k * D + d);
      }
    }
  }
  if (a.cost_out) a.cost_out[b] = cost;
  if (a.status) a.status[b] = st;
  if (a.n_free_out) a.n_free_out[b] = n_free;
}

template <int N, int R>
hipError_t launch_split_nr(const SolveArgs& a, double* ws, hipStream_t stream) {
  const int64_t V = a.K + 1;
  const int64_t n1 = a.B * V;
  if (a.B == 0) return hipSuccess;
  hipLaunchKernelGGL((assemble_kernel<N, R>), dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, stream, a, ws);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((block_cholesky_kernel<N, R>), dim3((unsigned)((a.B + 127) / 128)), dim3(128), 0, stream, a,
                     ws);
  return hipGetLastError();
}

template <int N>
hipError_t launch_split_n(const SolveArgs& a, double* ws, hipStream_t stream) {
  switch (a.r) {
    case 0: return launch_split_nr<N, 0>(a, ws, stream);
    case 1: if constexpr (N / 2 > 1) return launch_split_nr<N, 1>(a, ws, stream); break;
    case 2: if constexpr (N / 2 > 2) return launch_split_nr<N, 2>(a, ws, stream); break;
    case 3: if constexpr (N / 2 > 3) return launch_split_nr<N, 3>(a, ws, stream); break;
    case 4: if constexpr (N / 2 > 4) return launch_split_nr<N, 4>(a, ws, stream); break;
    case 5: if constexpr (N / 2 > 5) return launch_split_nr<N, 5>(a, ws, stream); break;
    default: break;
  }
  return hipErrorInvalidValue;
}

}  // namespace split

size_t split_workspace_bytes(int N, int D, int K, int64_t B) {
  const int H = N / 2;
  return sizeof(double) * (size_t)(K + 1) * split::ws_elems(H, D) * (size_t)B;
}

hipError_t launch_solve_split(int N, const SolveArgs& a, void* workspace, hipStream_t stream) {
  using namespace split;
  double* ws = static_cast<double*>(workspace);
  switch (N) {
    case 2: return launch_split_n<2>(a, ws, stream);
    case 4: return launch_split_n<4>(a, ws, stream);
    case 6: return launch_split_n<6>(a, ws, stream);
    case 8: return launch_split_n<8>(a, ws, stream);
    case 10: return launch_split_n<10>(a, ws, stream);
    case 12: return launch_split_n<12>(a, ws, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
