// mtg_solve_reg.hip -- register-resident block-Thomas solve for K <= kRegKMax segments.
//
// Same algorithm and numerics as the general kernel in mtg_kernels.hip (symmetric pinning of
// the fixed derivatives, exact-rational Htilde / A(1)^-1 tables, block Thomas with h x h LDL^T
// factors, translation-relative fixed positions; DESIGN.md "Algorithm"), re-laid out for
// occupancy and instruction count on CDNA4:
// * The back-substitution operands are not kept in LDS.  Column lane c keeps column c of
//   G_v = S_v^-1 E_v for every vertex in registers (the vertex loop is unrolled to the
//   compile-time bound KMAX so the register array is statically indexed), and the dimension
//   lanes write x^_v = x_f,v + z_v over the vertex's own staged values in LDS, which the
//   forward sweep has already consumed.  LDS per trajectory is V h D + 8 h' doubles (1.7 KB for
//   N=10, K=10, D=3) instead of 3.6 KB, so occupancy is bounded by registers (2 waves/SIMD).
// * A wave's trajectories' vertex values are staged into LDS once, with coalesced loads.
// * Column lanes read their columns of Htilde (H is symmetric, so each column is a contiguous
//   row of the LDS copy) instead of forming mat-vecs with unit vectors; only BL g_{v-1} is a
//   true mat-vec for them.
// * Wave-uniform structure is used through scalar branches: when every trajectory of the wave
//   has the same masks at v-1, v, v+1 (all of the reference's generators, and any batch of one
//   mission profile), mat-vec columns that multiply zeros in every lane are skipped, and so are
//   pivots pinned in every trajectory (ends fixed to SNAP: the whole vertex).  Mixed masks take
//   the dense path, with the same results.
#include "mtg_device.h"

#include <stdlib.h>

namespace mtg {

constexpr int kRegKMax = 12;  // largest K served by the register-resident kernel

__host__ __device__ constexpr int even_up(int h) { return (h + 1) & ~1; }

// Per-trajectory stride of the exchange buffer: LG columns of h' = even(h) doubles, plus one so
// that the 4 trajectories of a half-wave fall on different LDS banks (ds_read2_b64 / ds_write
// banks are (a/4) mod 32: an even stride of 48 doubles put all four on the same banks).
__host__ __device__ constexpr int xs_stride(int H, int LG) { return LG * even_up(H) + 1; }

// LDS doubles per block: Htilde(N, r) copy, X [tpb][V h D], exchange [tpb][xs_stride],
// times [tpb][K], masks [tpb][V] bytes.
__host__ __device__ inline int reg_lds_doubles(int N, int D, int K, int LG) {
  const int H = N / 2, tpb = kBlock / LG;
  return N * N + tpb * ((K + 1) * H * D + xs_stride(H, LG) + K) + (tpb * (K + 1) + 7) / 8;
}

// T^c for this lane's column c (same bits as s[c]).
template <int H>
__device__ __forceinline__ double lane_power(const double (&s)[H], int c) {
  double p = s[0];
#pragma unroll
  for (int k = 1; k < H; ++k) {
    p = (c == k) ? s[k] : p;
    asm volatile("" : "+v"(p));  // keep the selects: LLVM would rebuild s[c] as a scratch array
  }
  return p;
}

// dst[i] = src[i], i < n, by one wave: lane-strided, in batches of U loads per lane that are all
// issued before the batch's LDS stores.
template <typename T, int U>
__device__ __forceinline__ void copy_to_lds(const T* src, T* dst, int n, int lane) {
  for (int base = 0; base < n; base += U * kBlock) {
    T r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * kBlock + lane;
      r[u] = src[i < n ? i : n - 1];  // clamped: unconditional loads stay in registers
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // unconditional too (out-of-range lanes rewrite dst[n-1] with the same value): a guarded
      // store would let the compiler sink each load into its branch, one HBM latency per load
      const int i = base + u * kBlock + lane;
      dst[i < n ? i : n - 1] = r[u];
    }
  }
}

// x[k] = X[v][k][d] where bit k of m is set, else 0 (m == 0 for non-dimension lanes).
template <int H>
__device__ __forceinline__ void load_x(const double* X, int v, int D, int d, unsigned m, double (&x)[H]) {
  const double* p = X + (v * H) * D + d;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const double t = p[k * D];
    x[k] = ((m >> k) & 1u) ? t : 0.0;
  }
}

// Factor the pinned h x h S_v gathered from the exchange buffer (column j at xs[j * HP]) and
// solve S_v x = rhs.  PIN = derivatives pinned in every trajectory of the wave (their rows and
// columns are the identity and their right-hand side is 0): those pivots are skipped at compile
// time.  Other pinned rows (per trajectory) are identity rows in S and factor trivially.
template <int H, int HP, unsigned PIN>
__device__ __forceinline__ void factor_solve(const double* xs, const double (&rhs)[H], double (&x)[H],
                                             double& pmin) {
  double S[H][H];
#pragma unroll
  for (int i = 0; i < H; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j)
      if (!((PIN >> i) & 1u) && !((PIN >> j) & 1u)) S[i][j] = xs[j * HP + i];
  double dg[H], dinv[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    if ((PIN >> j) & 1u) continue;
    double w[H];
    double dj = S[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) {
      if ((PIN >> k) & 1u) continue;
      w[k] = S[j][k] * dg[k];
      dj -= S[j][k] * w[k];
    }
    pmin = dj < pmin ? dj : pmin;
    const double inv = rcp(dj);
    dg[j] = dj;
    dinv[j] = inv;
#pragma unroll
    for (int i = j + 1; i < H; ++i) {
      if ((PIN >> i) & 1u) continue;
      double t = S[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) {
        if ((PIN >> k) & 1u) continue;
        t -= S[i][k] * w[k];
      }
      S[i][j] = t * inv;
    }
  }
  double y[H];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    if ((PIN >> i) & 1u) continue;
    double t = rhs[i];
#pragma unroll
    for (int k = 0; k < i; ++k) {
      if ((PIN >> k) & 1u) continue;
      t -= S[i][k] * y[k];
    }
    y[i] = t;
  }
#pragma unroll
  for (int i = H - 1; i >= 0; --i) {
    if ((PIN >> i) & 1u) {
      x[i] = 0.0;
      continue;
    }
    double t = y[i] * dinv[i];
#pragma unroll
    for (int k = i + 1; k < H; ++k) {
      if ((PIN >> k) & 1u) continue;
      t -= S[k][i] * x[k];
    }
    x[i] = t;
  }
}

// Per-vertex scalars of the forward sweep (wave-uniform flags and this lane's segment scalings).
template <int H>
struct VertexIn {
  bool has_prev, has_next;
  unsigned mp, mc, mn;  // this trajectory's masks at v-1, v, v+1
  unsigned xc1, xn1;    // fixed derivatives > 0 in any trajectory of the wave, at v and v+1
  bool skip_bl0;        // BL column 0 multiplies zero in every lane
  double xfp0;          // fixed position at v-1 (dimension lanes)
  double scp, spc;      // segment v-1: T^(1-2r), T^c
  double scn, snc;      // segment v:   T^(1-2r), T^c
};

// One forward block-Thomas step at vertex v (see solve_fused_kernel for the block equations):
// assemble this lane's column of S_v (column lanes) or right-hand side (dimension lanes), exchange
// the S columns through LDS, factor and solve.  PIN = derivatives pinned at v in every trajectory
// of the wave: their rows are skipped at compile time.  Out: x = column c of G_v (column lanes) or
// z_v (dimension lanes), 0 on pinned rows.
template <int N, int R, unsigned PIN>
__device__ __forceinline__ void vertex_solve(const VertexIn<N / 2>& in, bool is_g, bool is_d, int c, int cg,
                                             const double (&gp)[N / 2], const double (&xfc)[N / 2],
                                             const double (&xfn)[N / 2], const double (&sp)[N / 2],
                                             const double (&sn)[N / 2], const double* rowBT, const double* rowTL,
                                             cdouble* BLbase, cdouble* Hbase, double* xs, double (&x)[N / 2],
                                             double& pmin) {
  constexpr int H = N / 2;
  constexpr int HP = even_up(H);
  const bool c_free = is_g && !((in.mc >> cg) & 1u);
  const bool c_free_n = is_g && in.has_next && !((in.mn >> cg) & 1u);

  // per-lane inputs: a2 = -g_{v-1} (column lanes) or x^_{v-1} (dimension lanes);
  // a1 = x_f,v and a3 = x_f,v+1 (dimension lanes; zero in column lanes)
  double a2[H], a1b[H], a1t[H], a3[H];
#pragma unroll
  for (int k = 0; k < H; ++k) a2[k] = gp[k], a1b[k] = xfc[k], a1t[k] = xfc[k], a3[k] = xfn[k];
  if (R >= 1) {  // translation-relative positions (solve_fused_kernel, DESIGN.md "Numerics")
    const bool tp = in.has_prev && (in.mp & in.mc & 1u);
    const bool tn = in.has_next && (in.mc & in.mn & 1u);
    a1b[0] = tp ? xfc[0] - in.xfp0 : a1b[0];
    a2[0] = tp ? 0.0 : a2[0];
    a3[0] = tn ? xfn[0] - xfc[0] : a3[0];
    a1t[0] = tn ? 0.0 : a1t[0];
  }

  double out[H], yy[H];
#pragma unroll
  for (int i = 0; i < H; ++i) out[i] = 0.0, yy[i] = 0.0;
  if (in.has_prev) {  // bottom rows of H_{v-1}: BL a2 + BR a1
    cdouble* BL = launder((const double*)BLbase);
    double t[H];
    // lane column of BR: column c (column lanes, if free at v) or 0 (dimension lanes, x_f,v[0])
    const double kb = is_g ? (c_free ? in.spc : 0.0) : a1b[0];
#pragma unroll
    for (int i = 0; i < H; ++i)
      if (!((PIN >> i) & 1u)) t[i] = rowBT[H + i] * kb;
    if (!in.skip_bl0) {
#pragma unroll
      for (int i = 0; i < H; ++i)
        if (!((PIN >> i) & 1u)) t[i] += BL[i * H] * a2[0];
    }
#pragma unroll
    for (int j = 1; j < H; ++j) {
      const double uj = sp[j] * a2[j];
#pragma unroll
      for (int i = 0; i < H; ++i)
        if (!((PIN >> i) & 1u)) t[i] += BL[i * H + j] * uj;
    }
    if (in.xc1) {
      cdouble* Hs = launder((const double*)Hbase);
#pragma unroll
      for (int j = 1; j < H; ++j) {
        if (!((in.xc1 >> j) & 1u)) continue;
        const double uj = sp[j] * a1b[j];
#pragma unroll
        for (int i = 0; i < H; ++i)
          if (!((PIN >> i) & 1u)) t[i] += Hs[(H + i) * N + H + j] * uj;
      }
    }
#pragma unroll
    for (int i = 0; i < H; ++i)
      if (!((PIN >> i) & 1u)) out[i] = (in.scp * sp[i]) * t[i];
  }
  if (in.has_next) {  // top rows of H_v: TL a1 + TR a3 (+ the G right-hand side: TR column c)
    double t[H], y[H];
    const double kt = is_g ? (c_free ? in.snc : 0.0) : a1t[0];
    const double kyg = c_free_n ? in.snc : 0.0;  // column lanes: G right-hand side
    const double kyd = is_g ? 0.0 : a3[0];       // dimension lanes: TR x_f,v+1[0]
#pragma unroll
    for (int i = 0; i < H; ++i) {
      if ((PIN >> i) & 1u) continue;
      const double r = rowBT[i];
      t[i] = rowTL[i] * kt + r * kyd;
      y[i] = r * kyg;
    }
    if (in.xc1 | in.xn1) {
      cdouble* Hs = launder((const double*)Hbase);
#pragma unroll
      for (int j = 1; j < H; ++j) {
        if (!((in.xc1 >> j) & 1u)) continue;
        const double wj = sn[j] * a1t[j];
#pragma unroll
        for (int i = 0; i < H; ++i)
          if (!((PIN >> i) & 1u)) t[i] += Hs[i * N + j] * wj;
      }
#pragma unroll
      for (int j = 1; j < H; ++j) {
        if (!((in.xn1 >> j) & 1u)) continue;
        const double wj = sn[j] * a3[j];
#pragma unroll
        for (int i = 0; i < H; ++i)
          if (!((PIN >> i) & 1u)) t[i] += Hs[i * N + H + j] * wj;
      }
    }
#pragma unroll
    for (int i = 0; i < H; ++i) {
      if ((PIN >> i) & 1u) continue;
      const double f = in.scn * sn[i];
      out[i] += f * t[i];
      yy[i] = f * y[i];
    }
  }

  // column lanes: S column c (pinned rows 0; pinned column: e_c); all lanes: the right-hand side
  // of their solve, G_v (column lanes: TR column c) or z_v (dimension lanes: -out), 0 on fixed rows
  const double dflag = is_d ? 1.0 : 0.0;
  double rhs[H];
#pragma unroll
  for (int i = 0; i < H; ++i) {
    if ((PIN >> i) & 1u) {
      rhs[i] = 0.0;
      continue;
    }
    const double fm = ((in.mc >> i) & 1u) ? 0.0 : 1.0;
    const double o = fm * out[i];
    double sv = c_free ? o : (i == c ? 1.0 : 0.0);
    asm volatile("" : "+v"(sv));
    xs[c * HP + i] = sv;  // only column lanes' slots are read
    rhs[i] = fm * yy[i] - dflag * o;
  }
  __syncthreads();
  factor_solve<H, HP, PIN>(xs, rhs, x, pmin);
  __syncthreads();
}

// Forward block-Thomas sweep over vertices 0..K, unrolled at compile time up to KMAX by template
// recursion: step<V> returns early once V > K.  (A `for` loop with a `continue` guard unrolls too,
// but makes every step a merge point of the whole loop-carried state, which the register allocator
// pays for with ~70 register copies per vertex.)  G is statically indexed, so it stays in registers.
template <int N, int R, int KMAX>
struct Forward {
  static constexpr int H = N / 2;
  static constexpr unsigned HM = (1u << H) - 1u;
  // context (per lane, constant over the sweep)
  int K, D, d;
  bool is_g, is_d;
  int c, cg;
  double gsign, tscale;
  double* X;
  double* xs;
  const double* tms;
  const uint8_t* msk;
  const double* rowBT;
  const double* rowTL;
  cdouble* BLbase;
  cdouble* Hbase;
  // loop-carried state
  int st = 0, n_free = 0;
  double pmin = DBL_MAX;
  uint32_t pin_cls = 0;  // per vertex, 2 bits: 0 none / 1 {position} / 2 all / 3 other, fixed in
                         // every trajectory of the wave (wave-uniform)
  double G[KMAX][H];     // column lanes: column c of G_v, v < K
  double gp[H], xfc[H], xfn[H];
  double sp[H], sn[H];
  double scp = 0.0, scn = 0.0, spc = 0.0, snc = 0.0, xfp0 = 0.0;
  unsigned mp = 0, mc = 0, mn = 0;

  __device__ __forceinline__ void init() {
#pragma unroll
    for (int k = 0; k < H; ++k) gp[k] = 0.0, sp[k] = 0.0;
    const double T0 = tms[0] * tscale;
    if (!time_ok(T0)) st |= MTG_TRAJ_BAD_TIME;
    seg_powers<H, R>(T0, sn, scn);
    snc = lane_power<H>(sn, cg);
    unsigned raw = msk[0];
    if (raw & ~HM) st |= MTG_TRAJ_WARN_DROPPED;
    mc = raw & HM;
    raw = msk[1];
    if (raw & ~HM) st |= MTG_TRAJ_WARN_DROPPED;
    mn = raw & HM;
    load_x<H>(X, 0, D, d, is_d ? mc : 0u, xfc);
    load_x<H>(X, 1, D, d, is_d ? mn : 0u, xfn);
  }

  template <int V>
  __device__ __forceinline__ void step() {
    if constexpr (V <= KMAX) {
      if (V > K) return;
      const bool has_prev = V > 0, has_next = V < K;

      // wave-uniform masks (scalar): identical masks in all lanes enable the skips below
      const unsigned mm = mp | (mc << 8) | (mn << 16);
      const unsigned u = __builtin_amdgcn_readfirstlane(mm);
      const bool uni = __builtin_amdgcn_ballot_w64(mm != u) == 0;
      const unsigned uc = (u >> 8) & HM, un = (u >> 16) & HM;
      const unsigned pin = uni ? uc : 0u;
      pin_cls |= (pin == 0u ? 0u : pin == 1u ? 1u : pin == HM ? 2u : 3u) << (2 * V);

      double x[H];
#pragma unroll
      for (int i = 0; i < H; ++i) x[i] = 0.0;
      // pin == HM: every derivative fixed at v in every trajectory, S_v = I and rhs = 0, so x = 0
      if (pin != HM) {
        // fixed derivatives other than the position, in any trajectory of the wave, at v / v+1:
        // their columns of BR, TL, TR enter the dimension lanes' products through scalar loads
        const unsigned xc1 = (uni ? uc : HM) & ~1u, xn1 = (uni ? un : HM) & ~1u;
        // position fixed at v-1 and v in every trajectory: the BL column 0 term is zero in all lanes
        const bool skip_bl0 = uni && R >= 1 && has_prev && ((u & uc) & 1u);
        VertexIn<H> in{has_prev, has_next, mp, mc, mn, xc1, xn1, skip_bl0, xfp0, scp, spc, scn, snc};
        if (pin == 1u)
          vertex_solve<N, R, 1u>(in, is_g, is_d, c, cg, gp, xfc, xfn, sp, sn, rowBT, rowTL, BLbase, Hbase, xs, x,
                                 pmin);
        else
          vertex_solve<N, R, 0u>(in, is_g, is_d, c, cg, gp, xfc, xfn, sp, sn, rowBT, rowTL, BLbase, Hbase, xs, x,
                                 pmin);
      }
      if constexpr (V < KMAX) {
        if (has_next) {
#pragma unroll
          for (int i = 0; i < H; ++i) G[V][i] = x[i];
        }
      }
      if (is_d && pin != HM) {
#pragma unroll
        for (int i = 0; i < H; ++i)
          if (!(((pin == 1u ? 1u : 0u) >> i) & 1u)) X[(V * H + i) * D + d] = xfc[i] + x[i];
      }
#pragma unroll
      for (int i = 0; i < H; ++i) gp[i] = __builtin_fma(gsign, x[i], xfc[i]);  // -g (xfc = 0) or x^
      n_free += __builtin_popcount(~mc & HM);
      if (!has_next) return;
      xfp0 = xfc[0];
      mp = mc;
#pragma unroll
      for (int k = 0; k < H; ++k) sp[k] = sn[k], xfc[k] = xfn[k];
      scp = scn;
      spc = snc;
      mc = mn;
      if (V + 1 < K) {
        const double Tn = tms[V + 1] * tscale;
        if (!time_ok(Tn)) st |= MTG_TRAJ_BAD_TIME;
        seg_powers<H, R>(Tn, sn, scn);
        snc = lane_power<H>(sn, cg);
        const unsigned raw = msk[V + 2];
        if (raw & ~HM) st |= MTG_TRAJ_WARN_DROPPED;
        mn = raw & HM;
        load_x<H>(X, V + 2, D, d, is_d ? mn : 0u, xfn);
      } else {
        mn = 0;
#pragma unroll
        for (int k = 0; k < H; ++k) xfn[k] = 0.0;
      }
      step<V + 1>();
    }
  }
};

template <int N, int R, int KMAX>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2))) void solve_reg_kernel(
    SolveArgs a, int lg_log2) {
  constexpr int H = N / 2;
  constexpr int HP = even_up(H);
  constexpr unsigned HM = (1u << H) - 1u;
  extern __shared__ __attribute__((aligned(16))) double lds[];

  const int LG = 1 << lg_log2;
  const int lane = threadIdx.x;
  const int slot = lane >> lg_log2;
  const int c = lane & (LG - 1);
  const int tpb = kBlock >> lg_log2;
  const int K = a.K, V = K + 1, D = a.D;
  const int xsz = V * H * D;
  const int xss = xs_stride(H, LG);
  const int64_t pair0 = (int64_t)blockIdx.x * tpb;
  const int64_t pair = pair0 + slot;
  const bool valid = pair < a.B;
  const int64_t pb = valid ? pair : 0;
  const double tscale = a.scales ? a.scales[pb % a.n_cand] : 1.0;
  const bool is_g = c < H;
  const bool is_d = (c >= H) && (c < H + D);
  const int d = is_d ? c - H : 0;
  const int cg = is_g ? c : 0;
  const double gsign = is_g ? -1.0 : 1.0;

  double* ht = lds;                                   // Htilde(N, R), row-major N x N
  double* xall = lds + N * N;                         // [tpb][V][H][D]
  double* xsall = xall + tpb * xsz;                   // [tpb][xss] exchange
  double* tall = xsall + tpb * xss;                   // [tpb][K] segment times
  uint8_t* mall = reinterpret_cast<uint8_t*>(tall + tpb * K);  // [tpb][V] masks
  double* X = xall + slot * xsz;                      // values -> x^ -> x
#ifdef MTG_PHASE_TIMING
  // debug builds only: per-phase s_memtime deltas written over free_out (scripts/phase_timing.py)
  uint64_t tph[5];
  tph[0] = __builtin_amdgcn_s_memtime();
#define MTG_PHASE(k) tph[k] = __builtin_amdgcn_s_memtime()
#else
#define MTG_PHASE(k) (void)0
#endif
  double* xs = xsall + slot * xss;                    // column c at xs[c * HP]
  const double* tms = tall + slot * K;
  const uint8_t* msk = mall + slot * V;

  // ---- stage Htilde and the wave's vertex values, times and masks into LDS (coalesced).  All of
  // a lane's loads are issued before its first LDS store (copy_to_lds), so the wave pays one HBM
  // latency, not one per load.
  {
    const double* hg = c_htilde + MTG_HTILDE_OFF(N, R);
    if (a.n_cand == 1 && pair0 + tpb <= a.B) {  // the wave's trajectories are contiguous
      const double* src = a.values + pair0 * xsz;
      const int n = tpb * xsz;
      const double* ts = a.times + pair0 * K;
      const uint8_t* ms = a.mask + pair0 * V;
      // small arrays first (their loads are in flight while the values are requested)
      double tv[2];
      uint8_t mv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = lane + u * kBlock;
        tv[u] = ts[i < tpb * K ? i : tpb * K - 1];
        mv[u] = ms[i < tpb * V ? i : tpb * V - 1];
      }
      double hv[(N * N + kBlock - 1) / kBlock];
#pragma unroll
      for (int u = 0; u < (N * N + kBlock - 1) / kBlock; ++u) {
        const int i = lane + u * kBlock;
        hv[u] = hg[i < N * N ? i : N * N - 1];
      }
      if (((reinterpret_cast<uintptr_t>(src) & 15u) == 0) && !(n & 1))
        copy_to_lds<double2, 16>(reinterpret_cast<const double2*>(src), reinterpret_cast<double2*>(xall), n / 2,
                                 lane);
      else
        copy_to_lds<double, 16>(src, xall, n, lane);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = lane + u * kBlock;
        tall[i < tpb * K ? i : tpb * K - 1] = tv[u];
        mall[i < tpb * V ? i : tpb * V - 1] = mv[u];
      }
#pragma unroll
      for (int u = 0; u < (N * N + kBlock - 1) / kBlock; ++u) {
        const int i = lane + u * kBlock;
        ht[i < N * N ? i : N * N - 1] = hv[u];
      }
      // (trailing slots beyond tpb * K or tpb * V of the small arrays: more than 2 per lane)
      for (int i = lane + 2 * kBlock; i < tpb * K; i += kBlock) tall[i] = ts[i];
      for (int i = lane + 2 * kBlock; i < tpb * V; i += kBlock) mall[i] = ms[i];
    } else {
      for (int i = lane; i < N * N; i += kBlock) ht[i] = hg[i];
      for (int s = 0; s < tpb; ++s) {
        int64_t ps = pair0 + s;
        if (ps >= a.B) ps = 0;
        const int64_t ts = ps / a.n_cand;
        copy_to_lds<double, 4>(a.values + ts * xsz, xall + s * xsz, xsz, lane);
        for (int i = lane; i < K; i += kBlock) tall[s * K + i] = a.times[ts * K + i];
        for (int i = lane; i < V; i += kBlock) mall[s * V + i] = a.mask[ts * V + i];
      }
    }
  }
  __syncthreads();
  MTG_PHASE(1);

  cdouble* const BLbase = (cdouble*)(c_hbl + MTG_HBL_OFF(N, R));
  cdouble* const Hbase = (cdouble*)(c_htilde + MTG_HTILDE_OFF(N, R));
  // the table columns this lane reads per vertex (H symmetric: columns are contiguous rows):
  // column lanes their own column c, dimension lanes column 0 (the position derivative)
  const double* rowBT = ht + (H + cg) * N;  // [TR col | BR col]
  const double* rowTL = ht + cg * N;        // [TL col | ...]

  // ---- forward sweep (see solve_fused_kernel for the block equations)
  Forward<N, R, KMAX> fw{K, D, d, is_g, is_d, c, cg, gsign, tscale, X, xs, tms, msk, rowBT, rowTL, BLbase, Hbase};
  fw.init();
  fw.template step<0>();
  int st = fw.st, n_free = fw.n_free;
  const double pmin = fw.pmin;
  const uint32_t pin_cls = fw.pin_cls;
  double (&G)[KMAX][H] = fw.G;
  double (&gp)[H] = fw.gp;
  if (!(pmin > 0.0 && pmin <= DBL_MAX)) st |= MTG_TRAJ_NOT_SPD;
  MTG_PHASE(2);

  // ---- backward substitution: x_v = x^_v - G_v x_{v+1} (dimension lanes; G_v via the exchange)
  double xn[H];
#pragma unroll
  for (int i = 0; i < H; ++i) xn[i] = gp[i];  // x_K = x^_K
#pragma unroll
  for (int v = KMAX - 1; v >= 0; --v) {
    if (v >= K) continue;
    const unsigned cls = (pin_cls >> (2 * v)) & 3u, clsn = (pin_cls >> (2 * v + 2)) & 3u;
    const unsigned pin = cls == 1u ? 1u : 0u, pinn = clsn == 1u ? 1u : 0u;  // rows/columns skipped
    if (cls == 2u || clsn == 2u) {  // G_v == 0: x_v = x^_v (already in X)
      if (is_d) {
#pragma unroll
        for (int i = 0; i < H; ++i) xn[i] = X[(v * H + i) * D + d];
      }
      continue;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < H; ++i)
      if (!((pin >> i) & 1u)) xs[c * HP + i] = G[v][i];
    __syncthreads();
    double x[H];
#pragma unroll
    for (int i = 0; i < H; ++i) x[i] = X[(v * H + i) * D + d];
#pragma unroll
    for (int cc = 0; cc < H; ++cc) {
      if ((pinn >> cc) & 1u) continue;
      const double xc = xn[cc];
#pragma unroll
      for (int i = 0; i < H; ++i)
        if (!((pin >> i) & 1u)) x[i] -= xs[cc * HP + i] * xc;
    }
    if (is_d) {
#pragma unroll
      for (int i = 0; i < H; ++i)
        if (!((pin >> i) & 1u)) X[(v * H + i) * D + d] = x[i];
    }
#pragma unroll
    for (int i = 0; i < H; ++i) xn[i] = x[i];
  }
  __syncthreads();
  MTG_PHASE(3);

  // ---- epilogue: coefficients and cost per item (segment i, dimension dd), spread over the group.
  // c = diag(T^-j) A(1)^-1 S(T) [x_i - p 1; x_{i+1} - p 1] + p e_0 with p = x_i[0] (the polynomial of
  // the translated end values is p(t) - p: only c_0 changes, and p_i no longer cancels against
  // p_{i+1} in c_j, j >= h).  A(1)^-1 is diag(1/j!) on top and dense below; its dense rows (without
  // column 0, which multiplies the translated zero) are read into registers once for all items:
  // the G registers are dead here.
  double A1b[H][N - 1];
  double A1d[H];
  {
    const double* Ai1 = c_a1inv + MTG_A1INV_OFF(N);
#pragma unroll
    for (int j = 0; j < H; ++j) {
      double t = Ai1[j * N + j];
      asm volatile("" : "+v"(t));
      A1d[j] = t;
#pragma unroll
      for (int q = 1; q < N; ++q) {
        double u = Ai1[(H + j) * N + q];
        asm volatile("" : "+v"(u));
        A1b[j][q - 1] = u;
      }
    }
  }
  double cacc = 0.0;
  int ii = c / D, dd = c - (c / D) * D;  // item it = ii * D + dd, advanced by LG per round
  for (int it = c; it < K * D; it += LG) {
    const int i = ii;
    const double T = tms[i] * tscale;
    double s[H], sc;
    seg_powers<H, R>(T, s, sc);
    double sh[N];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      sh[k] = s[k] * X[(i * H + k) * D + dd];
      sh[H + k] = s[k] * X[((i + 1) * H + k) * D + dd];
    }
    const double p0 = sh[0];
    sh[0] = 0.0;
    sh[H] -= p0;
    if (a.coeffs) {
      const double tinv = rcp(T);
      double outc[N];
      double tp = 1.0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        double acc;
        if (j < H) {
          acc = (j == 0) ? p0 : A1d[j] * sh[j];
        } else {
          acc = 0.0;
#pragma unroll
          for (int q = 1; q < N; ++q) acc += A1b[j - H][q - 1] * sh[q];
        }
        outc[j] = acc * tp;
        tp *= tinv;
      }
      if (valid) {
        double2* dst = reinterpret_cast<double2*>(a.coeffs + ((pb * K + i) * D + dd) * N);
#pragma unroll
        for (int j = 0; j < N / 2; ++j) dst[j] = make_double2(outc[2 * j], outc[2 * j + 1]);
      }
    }
    if (a.cost_out) {  // 0.5 c^T Q c = 0.5 sc sh^T Htilde sh  (translation-invariant for r >= 1)
      cdouble* Hl = launder((const double*)Hbase);
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
    dd += LG;
    while (dd >= D) dd -= D, ++ii;
  }
#ifdef MTG_PHASE_TIMING
  MTG_PHASE(4);
  if (a.free_out && valid && c == 0) {
    double* fo = a.free_out + pb * D * ((int64_t)V * H);
    for (int k = 0; k < 4; ++k) fo[k] = (double)(tph[k + 1] - tph[k]);
  }
  if (false) {
#else
  if (a.free_out && valid && is_d) {
#endif
    double* fo = a.free_out + (pb * D + d) * ((int64_t)V * H);
    int idx = 0;
    for (int v = 0; v < V; ++v) {
      const unsigned mv = msk[v] & HM;
#pragma unroll
      for (int k = 0; k < H; ++k)
        if (!((mv >> k) & 1u)) fo[idx++] = X[(v * H + k) * D + d];
    }
  }
  if (a.cost_out) {
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

// ---------------------------------------------------------------- dispatch
static int reg_kmax(int K) { return K <= 4 ? 4 : K <= 8 ? 8 : K <= 10 ? 10 : K <= kRegKMax ? kRegKMax : -1; }

bool reg_geometry(int N, int D, int K, int* lanes_per_traj, size_t* lds_bytes) {
  const int H = N / 2;
  // G_v columns take H * KMAX doubles per lane: beyond ~50 the kernel spills (N=12, K > 8)
  if (reg_kmax(K) < 0 || H * reg_kmax(K) > 50) return false;
  int lg = 8;
  while (lg < H + D) lg *= 2;
  if (lg > 64) return false;
  const size_t bytes = (size_t)reg_lds_doubles(N, D, K, lg) * sizeof(double);
  if (bytes > kMaxLdsPerBlock) return false;
  *lanes_per_traj = lg;
  *lds_bytes = bytes;
  return true;
}

template <int N, int R, int KMAX>
static hipError_t launch_reg_nrk(const SolveArgs& a, int lg, size_t lds, hipStream_t stream) {
  int lg_log2 = 0;
  while ((1 << lg_log2) < lg) ++lg_log2;
  const int tpb = kBlock / lg;
  const int64_t blocks = (a.B + tpb - 1) / tpb;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((solve_reg_kernel<N, R, KMAX>), dim3((unsigned)blocks), dim3(kBlock), lds, stream, a,
                     lg_log2);
  return hipGetLastError();
}

template <int N, int R>
static hipError_t launch_reg_nr(const SolveArgs& a, int lg, size_t lds, hipStream_t stream) {
  switch (reg_kmax(a.K)) {
    case 4: return launch_reg_nrk<N, R, 4>(a, lg, lds, stream);
    case 8: return launch_reg_nrk<N, R, 8>(a, lg, lds, stream);
    case 10: return launch_reg_nrk<N, R, 10>(a, lg, lds, stream);
    case kRegKMax: return launch_reg_nrk<N, R, kRegKMax>(a, lg, lds, stream);
    default: return hipErrorInvalidValue;
  }
}

template <int N>
static hipError_t launch_reg_n(const SolveArgs& a, int lg, size_t lds, hipStream_t stream) {
  switch (a.r) {
    case 0: return launch_reg_nr<N, 0>(a, lg, lds, stream);
    case 1: if constexpr (N / 2 > 1) return launch_reg_nr<N, 1>(a, lg, lds, stream); break;
    case 2: if constexpr (N / 2 > 2) return launch_reg_nr<N, 2>(a, lg, lds, stream); break;
    case 3: if constexpr (N / 2 > 3) return launch_reg_nr<N, 3>(a, lg, lds, stream); break;
    case 4: if constexpr (N / 2 > 4) return launch_reg_nr<N, 4>(a, lg, lds, stream); break;
    case 5: if constexpr (N / 2 > 5) return launch_reg_nr<N, 5>(a, lg, lds, stream); break;
    default: break;
  }
  return hipErrorInvalidValue;
}

hipError_t launch_solve_reg(int N, const SolveArgs& a, hipStream_t stream) {
  int lg;
  size_t lds;
  if (!reg_geometry(N, a.D, a.K, &lg, &lds)) return hipErrorInvalidValue;
  switch (N) {
    case 2: return launch_reg_n<2>(a, lg, lds, stream);
    case 4: return launch_reg_n<4>(a, lg, lds, stream);
    case 6: return launch_reg_n<6>(a, lg, lds, stream);
    case 8: return launch_reg_n<8>(a, lg, lds, stream);
    case 10: return launch_reg_n<10>(a, lg, lds, stream);
    case 12: return launch_reg_n<12>(a, lg, lds, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
