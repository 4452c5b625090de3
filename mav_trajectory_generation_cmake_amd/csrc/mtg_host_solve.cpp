// mtg_host_solve.cpp -- the host (CPU) solve path of the library: mtg_host_solve_linear_batch.
//
// The reference solves one problem at a time on the CPU (PolynomialOptimization<N>::solveLinear,
// lin_impl:329-369).  A single problem is a few microseconds of arithmetic, far below one GPU
// round trip (launch + two DMAs + synchronisation, ~40 us on MI355X), so a one-trajectory call
// (BASELINE config 1, the drop-in's most common call shape) is served here, on the calling
// thread.  Batches belong on the GPU (mtg_solve_linear_batch).
//
// This is product code, not the test oracle (oracle/ restates the reference's dense algorithm and
// is only a checker).  It is the same algorithm as the HIP kernels, in scalar C++:
// * exact-rational tables (gen_tables.py): H_i = T^(1-2r) S Htilde S, A_i^-1 = diag(T^-j) A(1)^-1 S,
//   S = diag(T^(slot mod h))  (updateSegmentTimes / computeQuadraticCostJacobian /
//   setupMappingMatrix / invertMappingMatrix, lin_impl:102-169, :276-295, :574-589);
// * unknowns ordered by (vertex, derivative) -- the reference's std::set order
//   (setupConstraintReorderingMatrix, lin_impl:172-250) -- so R = M^T H M (constructR, :298-326)
//   is block tridiagonal with h x h blocks and is never formed;
// * fixed derivatives pinned symmetrically (identity rows and columns, values moved to the right-
//   hand side), which is R_pp d_p = -R_pf d_f (:341-365) for any mask;
// * block LDL^T Thomas elimination, all D dimensions against one factorisation (:355-365);
// * recovery c_i = A_i^-1 [x_i; x_{i+1}] relative to the segment's start position, and the cost
//   0.5 sum c^T Q c (updateSegmentsFromCompactConstraints :253-273, computeCost :114-130).
// "lin_impl" = mav_trajectory_generation/include/mav_trajectory_generation/impl/
//              polynomial_optimization_linear_impl.h
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "mtg.h"
#include "mtg_host_threads.h"
#include "mtg_tables.inc"

namespace {

const double kA1inv[MTG_A1INV_SIZE] = {MTG_A1INV_VALUES};
const double kHtilde[MTG_HTILDE_SIZE] = {MTG_HTILDE_VALUES};

// T > 0 and finite (CHECK_GT(segment_time, 0), lin_impl:287)
inline bool time_ok(double T) { return T > 0.0 && T <= DBL_MAX; }
// Status bits of one segment time: BAD_TIME for T <= 0 or not finite; for 0 < T < DBL_EPSILON the
// reference's A(T) is singular (baseCoeffsWithTime keeps only the t = 0 entry, polynomial.h:225), so
// its solve is undefined there: NOT_SPD.
inline int32_t time_bits(double T) {
  return !time_ok(T) ? MTG_TRAJ_BAD_TIME : (T < DBL_EPSILON ? MTG_TRAJ_NOT_SPD : 0);
}

// Per-thread working storage of one trajectory (sized for the largest call seen).
struct Scratch {
  std::vector<double> G;   // [K][H][H]  G_v = S_v^-1 E_v (pinned)
  std::vector<double> Z;   // [V][D][H]  z_v, then the pinned solution y_v = x_v - xf_v
  std::vector<double> W;   // [K][D][N]  H_i [xf_i; xf_i+1] (fixed-value products per segment)
  std::vector<double> PW;  // [K][H]     segment powers T^k
  std::vector<double> SC;  // [K]        T^(1-2r)
};

template <int N>
struct HostSolve {
  static constexpr int H = N / 2;
  static constexpr unsigned HM = (1u << H) - 1u;

  // LDL^T of the leading n x n block of S (the free derivatives of a vertex; lower triangle used), in
  // place; returns the smallest pivot.  ldlt_solve_n solves with it.
  static double ldlt_n(double (&S)[H][H], double (&dinv)[H], int n) {
    double pmin = DBL_MAX;
    double dg[H];
    for (int j = 0; j < n; ++j) {
      double w[H];
      double dj = S[j][j];
      for (int k = 0; k < j; ++k) {
        w[k] = S[j][k] * dg[k];
        dj -= S[j][k] * w[k];
      }
      pmin = (dj < pmin || dj != dj) ? dj : pmin;  // a NaN pivot sticks (NOT_SPD)
      const double inv = 1.0 / dj;
      dg[j] = dj;
      dinv[j] = inv;
      for (int i = j + 1; i < n; ++i) {
        double t = S[i][j];
        for (int k = 0; k < j; ++k) t -= S[i][k] * w[k];
        S[i][j] = t * inv;
      }
    }
    return pmin;
  }

  static void ldlt_solve_n(const double (&S)[H][H], const double (&dinv)[H], double* x, int n) {
    double y[H];
    for (int i = 0; i < n; ++i) {
      double t = x[i];
      for (int k = 0; k < i; ++k) t -= S[i][k] * y[k];
      y[i] = t;
    }
    for (int i = n - 1; i >= 0; --i) {
      double t = y[i] * dinv[i];
      for (int k = i + 1; k < n; ++k) t -= S[k][i] * x[k];
      x[i] = t;
    }
  }

  // a vertex's D compressed vectors (its free entries first) to the full layout, pinned entries 0
  static void expand(double* zv, int D, unsigned m) {
    int fc[H], nc = 0;
    for (int k = 0; k < H; ++k)
      if (!((m >> k) & 1u)) fc[nc++] = k;
    for (int d = 0; d < D; ++d) {
      double* z = zv + (size_t)d * H;
      double full[H];
      for (int k = 0; k < H; ++k) full[k] = 0.0;
      for (int a = 0; a < nc; ++a) full[fc[a]] = z[a];
      for (int k = 0; k < H; ++k) z[k] = full[k];
    }
  }

  // c_i = diag(T^-j) A(1)^-1 S(T) [x_i - p 1; x_i+1 - p 1] + p e_0 with p = x_i[0] (the polynomial of
  // the translated end values is p(t) - p: only c_0 changes), and the cost 0.5 sum c^T Q c =
  // 0.5 T^(1-2r) sh^T Htilde sh (translation-invariant for r >= 1).  x_v = xf_v + y_v, where xf
  // are the fixed values (where mask bit k is set) and y (nullable: 0) the solved remainder
  // [V][D][H]; PW / SCl the segment powers T^k and T^(1-2r).  Returns the cost.
  static double recover(int D, int K, int r, const double* values, const uint8_t* mask, const double* times,
                        const double* Y, const double* PW, const double* SCl, double* coeffs, bool want_cost) {
    const double* Ht = kHtilde + MTG_HTILDE_OFF(N, r);
    const double* A1 = kA1inv + MTG_A1INV_OFF(N);
    double cost = 0.0;
    for (int i = 0; i < K; ++i) {
      const double* s = PW + (size_t)i * H;
      const double T = times[i];
      const unsigned m0 = mask ? mask[i] & HM : HM, m1 = mask ? mask[i + 1] & HM : HM;
      for (int d = 0; d < D; ++d) {
        double sh[N];
        for (int k = 0; k < H; ++k) {
          const double x0 = ((m0 >> k) & 1u) ? values[((size_t)i * H + k) * D + d] : 0.0;
          const double x1 = ((m1 >> k) & 1u) ? values[((size_t)(i + 1) * H + k) * D + d] : 0.0;
          const double y0 = Y ? Y[((size_t)i * D + d) * H + k] : 0.0;
          const double y1 = Y ? Y[((size_t)(i + 1) * D + d) * H + k] : 0.0;
          sh[k] = s[k] * (x0 + y0);
          sh[H + k] = s[k] * (x1 + y1);
        }
        const double p0 = sh[0];
        sh[0] = 0.0;
        sh[H] -= p0;
        if (coeffs) {
          double* c = coeffs + ((size_t)i * D + d) * N;
          const double tinv = 1.0 / T;
          double tp = 1.0;
          for (int j = 0; j < N; ++j) {
            double acc;
            if (j < H) {
              acc = j == 0 ? p0 : A1[j * N + j] * sh[j];
            } else {
              acc = 0.0;
              for (int q = 1; q < N; ++q) acc += A1[j * N + q] * sh[q];
            }
            c[j] = acc * tp;
            tp *= tinv;
          }
        }
        if (want_cost) {
          if (r == 0) sh[0] = p0, sh[H] += p0;
          double q = 0.0;
          for (int p = 0; p < N; ++p) {
            double row = 0.5 * Ht[p * N + p] * sh[p];
            for (int t = p + 1; t < N; ++t) row += Ht[p * N + t] * sh[t];
            q += sh[p] * row;
          }
          cost += SCl[i] * q;
        }
      }
    }
    return cost;
  }

  // One trajectory.  values [V][H][D], mask [V], times [K]; outputs as in mtg.h (nullable).
  static int32_t solve(int D, int K, int r, const double* values, const uint8_t* mask, const double* times,
                       double* coeffs, double* free_out, int32_t* n_free_out, double* cost_out, Scratch& sc) {
    const int V = K + 1;
    const double* Ht = kHtilde + MTG_HTILDE_OFF(N, r);
    sc.G.resize((size_t)K * H * H);
    sc.Z.resize((size_t)V * D * H);
    sc.W.resize((size_t)K * D * N);
    sc.PW.resize((size_t)K * H);
    sc.SC.resize(K);
    double* G = sc.G.data();
    double* Z = sc.Z.data();
    double* Wp = sc.W.data();
    double* PW = sc.PW.data();
    double* SCl = sc.SC.data();
    int32_t st = 0;
    auto m_of = [&](int v) -> unsigned {
      if (mask[v] & ~HM) st |= MTG_TRAJ_WARN_DROPPED;  // setupFromVertices drops them (lin_impl:74-95)
      return mask[v] & HM;
    };
    auto xf = [&](int v, int k, int d, unsigned m) -> double {
      return ((m >> k) & 1u) ? values[((size_t)v * H + k) * D + d] : 0.0;
    };

    // segment scalings and the fixed-value products W_i = H_i [xf_i; xf_i+1] per dimension; where
    // both end positions are fixed (r >= 1) the positions are taken relative to the segment start
    // (H_i [1 0..0 1 0..0]^T = 0), which removes the cancellation of H^TL p_i + H^TR p_i+1
    for (int i = 0; i < K; ++i) {
      const double T = times[i];
      st |= time_bits(T);  // CHECK_GT(segment_time, 0) (lin_impl:287)
      double* s = PW + (size_t)i * H;
      s[0] = 1.0;
      for (int k = 1; k < H; ++k) s[k] = s[k - 1] * T;
      SCl[i] = r == 0 ? T : 1.0 / (s[r] * s[r - 1]);
      const unsigned m0 = mask[i] & HM, m1 = mask[i + 1] & HM;
      const bool rel = r >= 1 && (m0 & m1 & 1u);
      for (int d = 0; d < D; ++d) {
        double u[N];
        for (int k = 0; k < H; ++k) {
          u[k] = s[k] * xf(i, k, d, m0);
          u[H + k] = s[k] * xf(i + 1, k, d, m1);
        }
        if (rel) {
          u[H] -= u[0];
          u[0] = 0.0;
        }
        // H u over the nonzero (fixed) entries of u only: interior waypoints fix just the position
        double* w = Wp + ((size_t)i * D + d) * N;
        double t[N];
        for (int a = 0; a < N; ++a) t[a] = 0.0;
        for (int b = 0; b < N; ++b) {
          if (u[b] == 0.0) continue;
          for (int a = 0; a < N; ++a) t[a] += Ht[a * N + b] * u[b];
        }
        for (int a = 0; a < N; ++a) w[a] = SCl[i] * s[a % H] * t[a];
      }
    }

    // forward sweep: S_v = D_v - E_{v-1}^T G_{v-1}, [G_v | z_v] = S_v^-1 [E_v | rhs_v], over the free
    // derivatives of each vertex only (fc[0..nc) at v, fp at v-1, fn at v+1): the pinned rows and
    // columns of the symmetric pinning are identity rows with a zero right-hand side, so they add
    // only exact zeros to the free entries' sums and their unknowns are 0 -- skipping them leaves
    // every free entry's arithmetic, in the same order, unchanged.  G_v is [nc][nn] and z_v [D][nc]
    // in the slots of the full layout; the solution is expanded to [V][D][H] afterwards.
    double pmin = DBL_MAX;
    int n_free = 0;
    unsigned mc = m_of(0);
    int fp[H], fc[H], fn[H], np_ = 0, nc = 0, nn = 0;
    for (int k = 0; k < H; ++k)
      if (!((mc >> k) & 1u)) fc[nc++] = k;
    for (int v = 0; v < V; ++v) {
      const unsigned mn = v < K ? m_of(v + 1) : HM;
      nn = 0;
      for (int k = 0; k < H; ++k)
        if (!((mn >> k) & 1u)) fn[nn++] = k;
      n_free += nc;
      double S[H][H];
      double Et[H][H];  // E_{v-1}^T on the free rows at v and free columns at v-1
      for (int i = 0; i < nc; ++i)
        for (int j = 0; j <= i; ++j) S[i][j] = 0.0;
      if (v > 0) {
        const double* s = PW + (size_t)(v - 1) * H;
        const double f = SCl[v - 1];
        for (int i = 0; i < nc; ++i)
          for (int j = 0; j <= i; ++j) S[i][j] += f * s[fc[i]] * s[fc[j]] * Ht[(H + fc[i]) * N + H + fc[j]];
        for (int i = 0; i < nc; ++i)
          for (int a = 0; a < np_; ++a) Et[i][a] = f * s[fc[i]] * s[fp[a]] * Ht[(H + fc[i]) * N + fp[a]];
        const double* Gp = G + (size_t)(v - 1) * H * H;  // Gp[a][j], a free at v-1, j free at v
        for (int i = 0; i < nc; ++i)
          for (int j = 0; j <= i; ++j) {
            double t = 0.0;
            for (int a = 0; a < np_; ++a) t += Et[i][a] * Gp[a * H + j];
            S[i][j] -= t;
          }
      }
      if (v < K) {
        const double* s = PW + (size_t)v * H;
        const double f = SCl[v];
        for (int i = 0; i < nc; ++i)
          for (int j = 0; j <= i; ++j) S[i][j] += f * s[fc[i]] * s[fc[j]] * Ht[fc[i] * N + fc[j]];
      }
      double dinv[H];
      const double pv = nc ? ldlt_n(S, dinv, nc) : 1.0;
      pmin = (pv < pmin || pv != pv) ? pv : pmin;  // a NaN pivot sticks (NOT_SPD)
      if (v < K) {  // G_v columns: E_v (top-right block of H_v) on the free rows and columns
        const double* s = PW + (size_t)v * H;
        const double f = SCl[v];
        double* Gv = G + (size_t)v * H * H;  // Gv[i][c]
        for (int c = 0; c < nn; ++c) {
          double col[H];
          for (int i = 0; i < nc; ++i) col[i] = f * s[fc[i]] * s[fn[c]] * Ht[fc[i] * N + H + fn[c]];
          ldlt_solve_n(S, dinv, col, nc);
          for (int i = 0; i < nc; ++i) Gv[i * H + c] = col[i];
        }
      }
      for (int d = 0; d < D; ++d) {
        double rhs[H];
        for (int i = 0; i < nc; ++i) {
          double t = 0.0;
          if (v > 0) t += Wp[((size_t)(v - 1) * D + d) * N + H + fc[i]];
          if (v < K) t += Wp[((size_t)v * D + d) * N + fc[i]];
          if (v > 0) {
            const double* zp = Z + ((size_t)(v - 1) * D + d) * H;
            for (int a = 0; a < np_; ++a) t += Et[i][a] * zp[a];
          }
          rhs[i] = -t;
        }
        ldlt_solve_n(S, dinv, rhs, nc);
        double* z = Z + ((size_t)v * D + d) * H;
        for (int i = 0; i < nc; ++i) z[i] = rhs[i];
      }
      mc = mn;
      np_ = nc;
      nc = nn;
      for (int k = 0; k < H; ++k) {
        fp[k] = fc[k];
        fc[k] = fn[k];
      }
    }
    if (!(pmin > 0.0 && pmin <= DBL_MAX)) st |= MTG_TRAJ_NOT_SPD;

    // backward substitution: y_v = z_v - G_v y_{v+1} (free entries), then the full layout with the
    // pinned entries 0, vertex by vertex from the end (y_{v+1} is still compressed when y_v needs it)
    {
      expand(Z + (size_t)K * D * H, D, mask[K] & HM);
      for (int v = K - 1; v >= 0; --v) {
        const unsigned mvv = mask[v] & HM, mnx = mask[v + 1] & HM;
        const int ncv = H - __builtin_popcount(mvv);
        const double* Gv = G + (size_t)v * H * H;
        int fnx[H], nnx = 0;
        for (int k = 0; k < H; ++k)
          if (!((mnx >> k) & 1u)) fnx[nnx++] = k;
        for (int d = 0; d < D; ++d) {
          double* y = Z + ((size_t)v * D + d) * H;
          const double* yn = Z + ((size_t)(v + 1) * D + d) * H;  // (already expanded)
          for (int i = 0; i < ncv; ++i) {
            double t = y[i];
            for (int c = 0; c < nnx; ++c) t -= Gv[i * H + c] * yn[fnx[c]];
            y[i] = t;
          }
        }
        expand(Z + (size_t)v * D * H, D, mvv);
      }
    }

    // recovery and cost per (segment, dimension): x_v = xf_v + y_v
    const double cost = recover(D, K, r, values, mask, times, Z, PW, SCl, coeffs, cost_out != nullptr);
    if (cost_out) *cost_out = cost;
    if (n_free_out) *n_free_out = n_free;
    if (free_out) {  // getFreeConstraints: per dimension, free (vertex, derivative) in sorted order
      for (int d = 0; d < D; ++d) {
        double* fo = free_out + (size_t)d * V * H;
        int idx = 0;
        for (int v = 0; v < V; ++v) {
          const unsigned m = mask[v] & HM;
          for (int k = 0; k < H; ++k)
            if (!((m >> k) & 1u)) fo[idx++] = Z[((size_t)v * D + d) * H + k];
        }
        for (; idx < V * H; ++idx) fo[idx] = 0.0;
      }
    }
    return st;
  }
};

typedef int32_t (*SolveFn)(int, int, int, const double*, const uint8_t*, const double*, double*, double*, int32_t*,
                           double*, Scratch&);

SolveFn solver_for(int N) {
  switch (N) {
    case 2: return &HostSolve<2>::solve;
    case 4: return &HostSolve<4>::solve;
    case 6: return &HostSolve<6>::solve;
    case 8: return &HostSolve<8>::solve;
    case 10: return &HostSolve<10>::solve;
    case 12: return &HostSolve<12>::solve;
    default: return nullptr;
  }
}

}  // namespace

extern "C" int mtg_host_default_threads(void) { return mtg::usable_cpus(); }

extern "C" int mtg_host_solve_linear_batch(int N, int D, int K, int derivative_to_optimize, int64_t batch,
                                           const double* values, const uint8_t* fixed_mask, const double* times,
                                           double* coeffs, double* free_out, int32_t* n_free_out,
                                           double* cost_out, int32_t* status, int threads) {
  if (N < 2 || N > 12 || (N % 2)) return MTG_ERR_UNSUPPORTED_N;
  if (derivative_to_optimize < 0 || derivative_to_optimize > N / 2 - 1) return MTG_ERR_BAD_DERIVATIVE;
  if (K < 1 || D < 1 || batch < 0) return MTG_ERR_SIZE_MISMATCH;
  if (batch == 0) return MTG_OK;
  if (!values || !fixed_mask || !times) return MTG_ERR_INVALID_ARGUMENT;
  const SolveFn fn = solver_for(N);
  const int h = N / 2, V = K + 1;
  const size_t sv = (size_t)V * h * D, sc = (size_t)K * D * N, sf = (size_t)D * V * h;
  auto one = [&](int64_t b, Scratch& s) {
    const int32_t st = fn(D, K, derivative_to_optimize, values + b * sv, fixed_mask + b * V, times + b * K,
                          coeffs ? coeffs + b * sc : nullptr, free_out ? free_out + b * sf : nullptr,
                          n_free_out ? n_free_out + b : nullptr, cost_out ? cost_out + b : nullptr, s);
    if (status) status[b] = st;
  };
  int nt = threads > 0 ? threads : mtg::usable_cpus();
  if (nt < 1) nt = 1;
  if ((int64_t)nt > batch) nt = (int)batch;
  if (nt == 1) {
    static thread_local Scratch s;  // no allocation per call on the drop-in's single-problem path
    for (int64_t b = 0; b < batch; ++b) one(b, s);
    return MTG_OK;
  }
  // trajectories are independent: a shared counter hands out chunks of 64
  std::atomic<int64_t> next{0};
  auto worker = [&] {
    Scratch s;
    for (;;) {
      const int64_t b0 = next.fetch_add(64);
      if (b0 >= batch) break;
      const int64_t b1 = b0 + 64 < batch ? b0 + 64 : batch;
      for (int64_t b = b0; b < b1; ++b) one(b, s);
    }
  };
  std::vector<std::thread> pool;
  pool.reserve(nt - 1);
  for (int t = 1; t < nt; ++t) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
  return MTG_OK;
}

namespace {

// segment powers T^k (k < h) and T^(1-2r), as the solvers form them
void seg_scalings(int N, int r, double T, double* s, double* sc) {
  const int H = N / 2;
  s[0] = 1.0;
  for (int k = 1; k < H; ++k) s[k] = s[k - 1] * T;
  *sc = r == 0 ? T : 1.0 / (s[r] * s[r - 1]);
}

double falling(int n, int i) {  // Polynomial::base_coefficients_(n, i) (src/polynomial.cpp:140-155)
  if (i < n) return 0.0;
  double out = 1.0;
  for (int k = i - n + 1; k <= i; ++k) out *= (double)k;
  return out;
}

}  // namespace

extern "C" int mtg_host_segment_matrices(int N, int derivative_to_optimize, double T, double* A, double* A_inv,
                                         double* Q, double* H) {
  if (N < 2 || N > 12 || (N % 2)) return MTG_ERR_UNSUPPORTED_N;
  const int r = derivative_to_optimize, h = N / 2;
  if (r < 0 || r > h - 1) return MTG_ERR_BAD_DERIVATIVE;
  if (!time_ok(T)) return MTG_ERR_INVALID_ARGUMENT;
  double s[6], sc;
  seg_scalings(N, r, T, s, &sc);
  if (A) {  // setupMappingMatrix (lin_impl:102-111) with baseCoeffsWithTime (polynomial.h:215-233)
    for (int i = 0; i < N * N; ++i) A[i] = 0.0;
    for (int k = 0; k < h; ++k) {
      A[k * N + k] = falling(k, k);
      A[(h + k) * N + k] = falling(k, k);
      double tp = T;
      for (int j = k + 1; j < N; ++j) {
        A[(h + k) * N + j] = falling(k, j) * tp;
        tp *= T;
      }
    }
  }
  if (A_inv) {  // diag(T^-j) A(1)^-1 S(T)
    const double* A1 = kA1inv + MTG_A1INV_OFF(N);
    const double tinv = 1.0 / T;
    double tp = 1.0;
    for (int j = 0; j < N; ++j) {
      for (int q = 0; q < N; ++q) A_inv[j * N + q] = A1[j * N + q] * s[q % h] * tp;
      tp *= tinv;
    }
  }
  if (Q) {  // computeQuadraticCostJacobian (lin_impl:574-589), the reference's factor 2 included
    for (int i = 0; i < N * N; ++i) Q[i] = 0.0;
    for (int col = 0; col < N - r; ++col)
      for (int row = 0; row < N - r; ++row) {
        const double e = (N - 1 - r) * 2 + 1 - row - col;
        Q[(N - 1 - row) * N + (N - 1 - col)] =
            falling(r, N - 1 - row) * falling(r, N - 1 - col) * std::pow(T, e) * 2.0 / e;
      }
  }
  if (H) {  // A^-T Q A^-1 = T^(1-2r) S Htilde S
    const double* Ht = kHtilde + MTG_HTILDE_OFF(N, r);
    for (int a = 0; a < N; ++a)
      for (int b = 0; b < N; ++b) H[a * N + b] = sc * s[a % h] * s[b % h] * Ht[a * N + b];
  }
  return MTG_OK;
}

extern "C" int mtg_host_coefficients_from_vertices_batch(int N, int D, int K, int64_t batch,
                                                         const double* vertex_values, const double* times,
                                                         double* coeffs, int threads) {
  if (N < 2 || N > 12 || (N % 2)) return MTG_ERR_UNSUPPORTED_N;
  if (K < 1 || D < 1 || batch < 0) return MTG_ERR_SIZE_MISMATCH;
  if (batch == 0) return MTG_OK;
  if (!vertex_values || !times || !coeffs) return MTG_ERR_INVALID_ARGUMENT;
  const int h = N / 2, V = K + 1;
  (void)threads;  // one problem per call in the drop-in; a batch goes to the GPU (mtg.h)
  std::vector<double> pw((size_t)K * h), scl(K);
  for (int64_t b = 0; b < batch; ++b) {
    const double* tb = times + b * K;
    for (int i = 0; i < K; ++i) seg_scalings(N, 0, tb[i], pw.data() + (size_t)i * h, &scl[i]);
    const double* vb = vertex_values + b * (int64_t)V * h * D;
    double* cb = coeffs + b * (int64_t)K * D * N;
    switch (N) {
      case 2: HostSolve<2>::recover(D, K, 0, vb, nullptr, tb, nullptr, pw.data(), scl.data(), cb, false); break;
      case 4: HostSolve<4>::recover(D, K, 0, vb, nullptr, tb, nullptr, pw.data(), scl.data(), cb, false); break;
      case 6: HostSolve<6>::recover(D, K, 0, vb, nullptr, tb, nullptr, pw.data(), scl.data(), cb, false); break;
      case 8: HostSolve<8>::recover(D, K, 0, vb, nullptr, tb, nullptr, pw.data(), scl.data(), cb, false); break;
      case 10: HostSolve<10>::recover(D, K, 0, vb, nullptr, tb, nullptr, pw.data(), scl.data(), cb, false); break;
      default: HostSolve<12>::recover(D, K, 0, vb, nullptr, tb, nullptr, pw.data(), scl.data(), cb, false); break;
    }
  }
  return MTG_OK;
}
