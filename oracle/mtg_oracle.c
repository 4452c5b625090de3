/*
 * mtg_oracle.c -- TEST INFRASTRUCTURE ONLY.  See mtg_oracle.h for the rules.
 *
 * A faithful, dependency-free C restatement of the reference CPU path.
 * "lin_impl" = mav_trajectory_generation/include/mav_trajectory_generation/
 *              impl/polynomial_optimization_linear_impl.h
 * All other paths are relative to the reference root.
 */
#include "mtg_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* std::mt19937 (C++ [rand.predef]; libstdc++ bits/random.tcc)              */
/* ------------------------------------------------------------------------ */
void oracle_mt_seed(oracle_mt19937* g, uint32_t seed) {
  g->mt[0] = seed;
  for (int i = 1; i < 624; ++i)
    g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
  g->idx = 624;
}

static void mt_twist(oracle_mt19937* g) {
  const uint32_t upper = 0x80000000u, lower = 0x7fffffffu;
  for (int k = 0; k < 624; ++k) {
    uint32_t y = (g->mt[k] & upper) | (g->mt[(k + 1) % 624] & lower);
    g->mt[k] = g->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  g->idx = 0;
}

uint32_t oracle_mt_next(oracle_mt19937* g) {
  if (g->idx >= 624) mt_twist(g);
  uint32_t z = g->mt[g->idx++];
  z ^= (z >> 11);
  z ^= (z << 7) & 0x9d2c5680u;
  z ^= (z << 15) & 0xefc60000u;
  z ^= (z >> 18);
  return z;
}

/* libstdc++ generate_canonical<double,53>(mt19937): k = 2 draws,
 * sum = g1 + g2*2^32 (in double), ret = sum / 2^64, clamp below 1;
 * uniform_real_distribution: ret * (b - a) + a. */
double oracle_uniform(oracle_mt19937* g, double a, double b) {
  double sum = 0.0, tmp = 1.0;
  for (int k = 0; k < 2; ++k) {
    sum += (double)oracle_mt_next(g) * tmp;
    tmp *= 4294967296.0;
  }
  double ret = sum / tmp;
  if (ret >= 1.0) ret = nextafter(1.0, 0.0);
  return ret * (b - a) + a;
}

/* Eigen's squaredNorm() summation order for a dynamic double vector with
 * SSE2 packets of 2 (Eigen/src/Core/Redux.h, LinearVectorizedTraversal):
 * for size <= 3 this is plain left-to-right. */
static double eigen_squared_norm(const double* x, int n) {
  if (n <= 0) return 0.0;
  int aligned2 = (n / 4) * 4, aligned = (n / 2) * 2;
  if (!aligned) return x[0] * x[0];
  double p0a = x[0] * x[0], p0b = x[1] * x[1];
  if (aligned > 2) {
    double p1a = x[2] * x[2], p1b = x[3] * x[3];
    for (int i = 4; i < aligned2; i += 4) {
      p0a += x[i] * x[i];
      p0b += x[i + 1] * x[i + 1];
      p1a += x[i + 2] * x[i + 2];
      p1b += x[i + 3] * x[i + 3];
    }
    p0a += p1a;
    p0b += p1b;
    if (aligned > aligned2) {
      p0a += x[aligned2] * x[aligned2];
      p0b += x[aligned2 + 1] * x[aligned2 + 1];
    }
  }
  double res = p0a + p0b;
  for (int i = aligned; i < n; ++i) res += x[i] * x[i];
  return res;
}

/* ------------------------------------------------------------------------ */
/* polynomial.h / src/polynomial.cpp                                        */
/* ------------------------------------------------------------------------ */
/* computeBaseCoefficients (src/polynomial.cpp:140-155), table sized
 * kMaxConvolutionSize = 22 (polynomial.h:49, src/polynomial.cpp:177-178). */
#define BASE_N 22
static double g_base[BASE_N][BASE_N];
static int g_base_init = 0;

static void base_init(void) {
  if (g_base_init) return;
  memset(g_base, 0, sizeof(g_base));
  for (int i = 0; i < BASE_N; ++i) g_base[0][i] = 1.0;
  const int DEG = BASE_N - 1;
  int order = DEG;
  for (int n = 1; n < BASE_N; ++n) {
    for (int i = DEG - order; i < BASE_N; ++i)
      g_base[n][i] = (double)(order - DEG + i) * g_base[n - 1][i];
    order--;
  }
  g_base_init = 1;
}

/* The table is filled once, before any parallel region reads it: a lazy first fill from inside an
 * OpenMP loop let one thread's memset run while another thread, seeing g_base_init already set,
 * read the half-rebuilt table (a fresh process's first multi-threaded call could return wrong
 * coefficients: one smoke run saw a 1.5 scale-normalised error against correct GPU results). */
__attribute__((constructor)) static void base_ctor(void) { base_init(); }

double oracle_base_coefficient(int n, int i) {
  base_init();
  if (n < 0 || i < 0 || n >= BASE_N || i >= BASE_N) return 0.0;
  return g_base[n][i];
}

/* Polynomial::baseCoeffsWithTime (polynomial.h:215-233), incl. the |t|<eps rule. */
void oracle_base_coeffs_with_time(int N, int derivative, double t, double* out) {
  base_init();
  for (int j = 0; j < N; ++j) out[j] = 0.0;
  out[derivative] = g_base[derivative][derivative];
  if (fabs(t) < DBL_EPSILON) return;
  double t_power = t;
  for (int j = derivative + 1; j < N; ++j) {
    out[j] = g_base[derivative][j] * t_power;
    t_power = t_power * t;
  }
}

/* Polynomial::evaluate(t, derivative) (polynomial.h:138-151): Horner. */
double oracle_poly_evaluate(int N, const double* c, double t, int derivative) {
  base_init();
  if (derivative >= N) return 0.0;
  const int tmp = N - 1;
  double result = g_base[derivative][tmp] * c[tmp];
  for (int j = tmp - 1; j >= derivative; --j) {
    result *= t;
    result += g_base[derivative][j] * c[j];
  }
  return result;
}

/* ------------------------------------------------------------------------ */
/* Generators                                                               */
/* ------------------------------------------------------------------------ */
static void make_start_or_end(int nd, int D, double* vvals, uint32_t* vmask, const double* pos,
                              int up_to) {
  /* Vertex::makeStartOrEnd (src/vertex.cpp:106-112) */
  for (int d = 0; d < D; ++d) vvals[0 * D + d] = pos[d];
  *vmask |= 1u;
  for (int k = 1; k <= up_to && k < nd; ++k) {
    for (int d = 0; d < D; ++d) vvals[k * D + d] = 0.0;
    *vmask |= (1u << k);
  }
}

/* createRandomVertices (src/vertex.cpp:27-79). */
int oracle_create_random_vertices(int max_derivative, int K, int D, const double* pos_min,
                                  const double* pos_max, uint32_t seed, int nd, double* values,
                                  uint32_t* mask) {
  if (K < 1 || D < 1 || max_derivative <= 0 || nd <= max_derivative || D > 64) return ORACLE_ERR_ARG;
  const int V = K + 1;
  memset(values, 0, sizeof(double) * (size_t)V * nd * D);
  memset(mask, 0, sizeof(uint32_t) * (size_t)V);
  oracle_mt19937 g;
  oracle_mt_seed(&g, seed);
  const double min_distance = 0.2;
  double last[64], pos[64], diff[64];
  for (int d = 0; d < D; ++d) last[d] = oracle_uniform(&g, pos_min[d], pos_max[d]);
  make_start_or_end(nd, D, values, &mask[0], last, max_derivative);
  for (int i = 1; i < V; ++i) {
    for (;;) {
      for (int d = 0; d < D; ++d) pos[d] = oracle_uniform(&g, pos_min[d], pos_max[d]);
      for (int d = 0; d < D; ++d) diff[d] = pos[d] - last[d];
      if (sqrt(eigen_squared_norm(diff, D)) > min_distance) break;
    }
    for (int d = 0; d < D; ++d) values[((size_t)i * nd + 0) * D + d] = pos[d];
    mask[i] |= 1u;
    for (int d = 0; d < D; ++d) last[d] = pos[d];
  }
  make_start_or_end(nd, D, values + (size_t)(V - 1) * nd * D, &mask[V - 1], last, max_derivative);
  return ORACLE_OK;
}

/* createRandomVerticesPath (src/polynomial_timing_evaluation.cpp:34-91),
 * including its quirk: last_position is set to the *offset* (:86) and the
 * final makeStartOrEnd(last_position) (:88) overwrites the last position. */
int oracle_create_random_vertices_path(int D, int K, double average_distance, int max_derivative,
                                       uint32_t seed, int nd, double* values, uint32_t* mask) {
  if (K < 1 || D < 1 || max_derivative <= 0 || nd <= max_derivative || D > 64) return ORACLE_ERR_ARG;
  const int V = K + 1;
  memset(values, 0, sizeof(double) * (size_t)V * nd * D);
  memset(mask, 0, sizeof(uint32_t) * (size_t)V);
  oracle_mt19937 g;
  oracle_mt_seed(&g, seed);
  const double min_distance = 0.2;
  double last[64], ps[64];
  for (int d = 0; d < D; ++d) last[d] = oracle_uniform(&g, -1.0, 1.0);
  make_start_or_end(nd, D, values, &mask[0], last, max_derivative);
  double distance_accumulated = 0.0;
  for (int i = 1; i < V; ++i) {
    for (;;) {
      for (int d = 0; d < D; ++d) ps[d] = oracle_uniform(&g, -1.0, 1.0);
      if (sqrt(eigen_squared_norm(ps, D)) > min_distance) break;
    }
    double z = eigen_squared_norm(ps, D);
    double s = sqrt(z);
    double dist = oracle_uniform(&g, 0.0, 2.0 * average_distance);
    for (int d = 0; d < D; ++d) ps[d] = (z > 0.0 ? ps[d] / s : ps[d]) * dist;
    distance_accumulated += sqrt(eigen_squared_norm(ps, D));
    for (int d = 0; d < D; ++d) values[((size_t)i * nd + 0) * D + d] = ps[d] + last[d];
    mask[i] |= 1u;
    for (int d = 0; d < D; ++d) last[d] = ps[d];
  }
  (void)distance_accumulated;
  make_start_or_end(nd, D, values + (size_t)(V - 1) * nd * D, &mask[V - 1], last, max_derivative);
  return ORACLE_OK;
}

/* estimateSegmentTimes (src/vertex.cpp:162-178). */
void oracle_estimate_segment_times(int K, int D, int nd, const double* values, double v_max,
                                   double a_max, double magic_fabian_constant, double* times) {
  double diff[64];
  for (int i = 0; i < K; ++i) {
    const double* s = values + (size_t)i * nd * D;
    const double* e = values + (size_t)(i + 1) * nd * D;
    for (int d = 0; d < D; ++d) diff[d] = e[d] - s[d];
    double distance = sqrt(eigen_squared_norm(diff, D));
    times[i] = distance / v_max * 2 *
               (1.0 + magic_fabian_constant * v_max / a_max * exp(-distance / v_max * 2));
  }
}

/* ------------------------------------------------------------------------ */
/* Dense helpers                                                            */
/* ------------------------------------------------------------------------ */
/* Inverse of an n x n matrix by LU with partial pivoting (stands in for
 * Eigen's fixed-size .inverse(), lin_impl:160-161). */
static void lu_inverse(int n, const double* A, double* Ainv) {
  double lu[ORACLE_KMAXN * ORACLE_KMAXN];
  int piv[ORACLE_KMAXN];
  memcpy(lu, A, sizeof(double) * n * n);
  for (int i = 0; i < n; ++i) piv[i] = i;
  for (int k = 0; k < n; ++k) {
    int p = k;
    double best = fabs(lu[k * n + k]);
    for (int i = k + 1; i < n; ++i)
      if (fabs(lu[i * n + k]) > best) best = fabs(lu[i * n + k]), p = i;
    if (p != k) {
      for (int j = 0; j < n; ++j) {
        double t = lu[k * n + j];
        lu[k * n + j] = lu[p * n + j];
        lu[p * n + j] = t;
      }
      int t = piv[k];
      piv[k] = piv[p];
      piv[p] = t;
    }
    for (int i = k + 1; i < n; ++i) {
      lu[i * n + k] /= lu[k * n + k];
      for (int j = k + 1; j < n; ++j) lu[i * n + j] -= lu[i * n + k] * lu[k * n + j];
    }
  }
  for (int c = 0; c < n; ++c) {
    double x[ORACLE_KMAXN];
    for (int i = 0; i < n; ++i) x[i] = (piv[i] == c) ? 1.0 : 0.0;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < i; ++j) x[i] -= lu[i * n + j] * x[j];
    for (int i = n - 1; i >= 0; --i) {
      for (int j = i + 1; j < n; ++j) x[i] -= lu[i * n + j] * x[j];
      x[i] /= lu[i * n + i];
    }
    for (int i = 0; i < n; ++i) Ainv[i * n + c] = x[i];
  }
}

/* Solve A x = b for an n x n dense A (row-major) by Householder QR; `nrhs`
 * right-hand sides stored as b[rhs][n].  Stands in for SparseQR (lin_impl:355-364). */
static void qr_solve(int n, double* A, int nrhs, double* b) {
  double* v = (double*)malloc(sizeof(double) * n);
  double* tau = (double*)malloc(sizeof(double) * n);
  for (int k = 0; k < n; ++k) {
    double norm = 0.0;
    for (int i = k; i < n; ++i) norm += A[i * n + k] * A[i * n + k];
    norm = sqrt(norm);
    double alpha = A[k * n + k] > 0 ? -norm : norm;
    for (int i = k; i < n; ++i) v[i] = A[i * n + k];
    v[k] -= alpha;
    double vnorm2 = 0.0;
    for (int i = k; i < n; ++i) vnorm2 += v[i] * v[i];
    tau[k] = vnorm2 > 0 ? 2.0 / vnorm2 : 0.0;
    for (int j = k; j < n; ++j) {
      double s = 0.0;
      for (int i = k; i < n; ++i) s += v[i] * A[i * n + j];
      s *= tau[k];
      for (int i = k; i < n; ++i) A[i * n + j] -= s * v[i];
    }
    for (int q = 0; q < nrhs; ++q) {
      double* bq = b + (size_t)q * n;
      double s = 0.0;
      for (int i = k; i < n; ++i) s += v[i] * bq[i];
      s *= tau[k];
      for (int i = k; i < n; ++i) bq[i] -= s * v[i];
    }
  }
  for (int q = 0; q < nrhs; ++q) {
    double* bq = b + (size_t)q * n;
    for (int i = n - 1; i >= 0; --i) {
      double s = bq[i];
      for (int j = i + 1; j < n; ++j) s -= A[i * n + j] * bq[j];
      bq[i] = s / A[i * n + i];
    }
  }
  free(v);
  free(tau);
}

/* ------------------------------------------------------------------------ */
/* PolynomialOptimization<N> statics                                        */
/* ------------------------------------------------------------------------ */
/* setupMappingMatrix (lin_impl:102-111). */
void oracle_setup_mapping_matrix(int N, double T, double* A) {
  const int h = N / 2;
  for (int i = 0; i < h; ++i) {
    oracle_base_coeffs_with_time(N, i, 0.0, A + (size_t)i * N);
    oracle_base_coeffs_with_time(N, i, T, A + (size_t)(i + h) * N);
  }
}

/* invertMappingMatrix (lin_impl:133-169): Schur complement of
 * [A_diag 0; C D]  ->  [A_diag^-1 0; -D^-1 C A_diag^-1  D^-1]. */
void oracle_invert_mapping_matrix(int N, const double* A, double* Ainv) {
  const int h = N / 2;
  double Dm[ORACLE_KMAXN * ORACLE_KMAXN / 4], Dinv[ORACLE_KMAXN * ORACLE_KMAXN / 4];
  double adiag_inv[ORACLE_KMAXN / 2];
  for (int i = 0; i < h; ++i) adiag_inv[i] = 1.0 / A[i * N + i];
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < h; ++j) Dm[i * h + j] = A[(i + h) * N + (j + h)];
  lu_inverse(h, Dm, Dinv);
  for (int i = 0; i < N * N; ++i) Ainv[i] = 0.0;
  for (int i = 0; i < h; ++i) Ainv[i * N + i] = adiag_inv[i];
  /* -D_inv * C * A_inv, evaluated left to right as Eigen does. */
  double DC[ORACLE_KMAXN * ORACLE_KMAXN / 4];
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < h; ++j) {
      double s = 0.0;
      for (int k = 0; k < h; ++k) s += -Dinv[i * h + k] * A[(k + h) * N + j];
      DC[i * h + j] = s;
    }
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < h; ++j) {
      Ainv[(i + h) * N + j] = DC[i * h + j] * adiag_inv[j];
      Ainv[(i + h) * N + (j + h)] = Dinv[i * h + j];
    }
}

/* computeQuadraticCostJacobian (lin_impl:574-589). */
void oracle_quadratic_cost_jacobian(int N, int derivative, double t, double* Q) {
  base_init();
  for (int i = 0; i < N * N; ++i) Q[i] = 0.0;
  for (int col = 0; col < N - derivative; col++) {
    for (int row = 0; row < N - derivative; row++) {
      double exponent = (N - 1 - derivative) * 2 + 1 - row - col;
      Q[(N - 1 - row) * N + (N - 1 - col)] = g_base[derivative][N - 1 - row] *
                                              g_base[derivative][N - 1 - col] * pow(t, exponent) *
                                              2.0 / exponent;
    }
  }
}

/* ------------------------------------------------------------------------ */
/* setupFromVertices + solveLinear                                          */
/* ------------------------------------------------------------------------ */
int oracle_solve_linear(const oracle_problem* p, oracle_outputs* out) {
  const int N = p->N, D = p->D, K = p->K, r = p->r, nd = p->nd;
  if (N < 2 || N > ORACLE_KMAXN || (N % 2) || D < 1 || K < 1 || nd < 1) return ORACLE_ERR_ARG;
  const int h = N / 2, V = K + 1;
  /* CHECK derivative_to_optimize (lin_impl:50-55) */
  if (r < 0 || r > h - 1) return ORACLE_ERR_BAD_DERIVATIVE;
  int ret = ORACLE_OK;

  /* Drop constraints of order > N/2-1 (lin_impl:74-95). */
  uint32_t* mask = (uint32_t*)malloc(sizeof(uint32_t) * V);
  for (int v = 0; v < V; ++v) {
    uint32_t m = p->mask[v];
    if (nd < 32) m &= (nd == 32 ? 0xffffffffu : ((1u << nd) - 1u));
    if (m >> h) ret |= ORACLE_WARN_DROPPED;
    mask[v] = m & ((1u << h) - 1u);
  }
  /* updateSegmentTimes (lin_impl:276-295). */
  double* Q = (double*)malloc(sizeof(double) * K * N * N);
  double* A = (double*)malloc(sizeof(double) * K * N * N);
  double* Ai = (double*)malloc(sizeof(double) * K * N * N);
  for (int i = 0; i < K; ++i) {
    const double T = p->times[i];
    if (!(T > 0.0)) { /* CHECK_GT(segment_time, 0) (lin_impl:287) */
      free(mask); free(Q); free(A); free(Ai);
      return ORACLE_ERR_BAD_TIME;
    }
    oracle_quadratic_cost_jacobian(N, r, T, Q + (size_t)i * N * N);
    oracle_setup_mapping_matrix(N, T, A + (size_t)i * N * N);
    oracle_invert_mapping_matrix(N, A + (size_t)i * N * N, Ai + (size_t)i * N * N);
  }

  /* setupConstraintReorderingMatrix (lin_impl:172-250).  Rows: vertices in
   * order, interior vertices twice, derivatives 0..h-1.  Columns: std::set
   * order (vertex, derivative) of fixed, then of free (Constraint::operator<,
   * polynomial_optimization_linear.h:272-289). */
  const int n_all = (2 * V - 2) * h;
  int* row_v = (int*)malloc(sizeof(int) * n_all);
  int* row_k = (int*)malloc(sizeof(int) * n_all);
  int row = 0;
  for (int v = 0; v < V; ++v) {
    int occ = (v == 0 || v == K) ? 1 : 2;
    for (int co = 0; co < occ; ++co)
      for (int k = 0; k < h; ++k) row_v[row] = v, row_k[row] = k, ++row;
  }
  int* col_fixed = (int*)malloc(sizeof(int) * V * h); /* (v,k) -> column */
  int n_fixed = 0, n_free = 0;
  for (int v = 0; v < V; ++v)
    for (int k = 0; k < h; ++k)
      if ((mask[v] >> k) & 1u) col_fixed[v * h + k] = n_fixed++;
  for (int v = 0; v < V; ++v)
    for (int k = 0; k < h; ++k)
      if (!((mask[v] >> k) & 1u)) col_fixed[v * h + k] = n_fixed + n_free++;
  const int n = n_fixed + n_free;
  int* col_of_row = (int*)malloc(sizeof(int) * n_all);
  for (int a = 0; a < n_all; ++a) col_of_row[a] = col_fixed[row_v[a] * h + row_k[a]];

  /* fixed_constraints_compact_ per dimension (lin_impl:228-237). */
  double* df = (double*)calloc((size_t)D * (n_fixed > 0 ? n_fixed : 1), sizeof(double));
  for (int v = 0; v < V; ++v)
    for (int k = 0; k < h; ++k)
      if ((mask[v] >> k) & 1u)
        for (int d = 0; d < D; ++d)
          df[(size_t)d * n_fixed + col_fixed[v * h + k]] = p->values[((size_t)v * nd + k) * D + d];
  double* dp = (double*)calloc((size_t)D * (n_free > 0 ? n_free : 1), sizeof(double));

  if (n_free > 0) {
    /* constructR (lin_impl:298-326): H_i = Ai^T Q Ai, R = M^T blkdiag(H) M. */
    double* R = (double*)calloc((size_t)n * n, sizeof(double));
    double tmp[ORACLE_KMAXN * ORACLE_KMAXN], H[ORACLE_KMAXN * ORACLE_KMAXN];
    for (int i = 0; i < K; ++i) {
      const double* ai = Ai + (size_t)i * N * N;
      const double* q = Q + (size_t)i * N * N;
      for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b) {
          double s = 0.0;
          for (int k = 0; k < N; ++k) s += ai[k * N + a] * q[k * N + b];
          tmp[a * N + b] = s;
        }
      for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b) {
          double s = 0.0;
          for (int k = 0; k < N; ++k) s += tmp[a * N + k] * ai[k * N + b];
          H[a * N + b] = s;
        }
      for (int a = 0; a < N; ++a)
        for (int b = 0; b < N; ++b)
          R[(size_t)col_of_row[i * N + a] * n + col_of_row[i * N + b]] += H[a * N + b];
    }
    /* Rpf, Rpp blocks and per-dimension solve (lin_impl:350-365). */
    double* Rpp = (double*)malloc(sizeof(double) * (size_t)n_free * n_free);
    for (int a = 0; a < n_free; ++a)
      for (int b = 0; b < n_free; ++b) Rpp[(size_t)a * n_free + b] = R[(size_t)(n_fixed + a) * n + n_fixed + b];
    for (int d = 0; d < D; ++d)
      for (int a = 0; a < n_free; ++a) {
        double s = 0.0;
        for (int b = 0; b < n_fixed; ++b) s += R[(size_t)(n_fixed + a) * n + b] * df[(size_t)d * n_fixed + b];
        dp[(size_t)d * n_free + a] = -s;
      }
    qr_solve(n_free, Rpp, D, dp);
    free(Rpp);
    free(R);
  }

  /* updateSegmentsFromCompactConstraints (lin_impl:253-273). */
  double* coeffs = (double*)malloc(sizeof(double) * (size_t)K * D * N);
  for (int d = 0; d < D; ++d) {
    for (int i = 0; i < K; ++i) {
      double nd_[ORACLE_KMAXN];
      for (int s = 0; s < N; ++s) {
        int c = col_of_row[i * N + s];
        nd_[s] = c < n_fixed ? df[(size_t)d * n_fixed + c] : dp[(size_t)d * n_free + (c - n_fixed)];
      }
      const double* ai = Ai + (size_t)i * N * N;
      for (int j = 0; j < N; ++j) {
        double s = 0.0;
        for (int k = 0; k < N; ++k) s += ai[j * N + k] * nd_[k];
        coeffs[((size_t)i * D + d) * N + j] = s;
      }
    }
  }
  if (out) {
    out->counts[0] = n_all;
    out->counts[1] = n_fixed;
    out->counts[2] = n_free;
    if (out->coeffs) memcpy(out->coeffs, coeffs, sizeof(double) * (size_t)K * D * N);
    if (out->fixed) memcpy(out->fixed, df, sizeof(double) * (size_t)D * n_fixed);
    if (out->free_) memcpy(out->free_, dp, sizeof(double) * (size_t)D * n_free);
    if (out->col_of_row) memcpy(out->col_of_row, col_of_row, sizeof(int) * n_all);
    if (out->ainv) memcpy(out->ainv, Ai, sizeof(double) * (size_t)K * N * N);
    if (out->amap) memcpy(out->amap, A, sizeof(double) * (size_t)K * N * N);
    if (out->qmat) memcpy(out->qmat, Q, sizeof(double) * (size_t)K * N * N);
    if (out->cost) {
      /* computeCost (lin_impl:114-130): 0.5 * sum c^T Q c. */
      double cost = 0.0;
      for (int i = 0; i < K; ++i)
        for (int d = 0; d < D; ++d) {
          const double* c = coeffs + ((size_t)i * D + d) * N;
          const double* q = Q + (size_t)i * N * N;
          double part = 0.0;
          for (int b = 0; b < N; ++b) {
            double cq = 0.0;
            for (int a = 0; a < N; ++a) cq += c[a] * q[a * N + b];
            part += cq * c[b];
          }
          cost += part;
        }
      *out->cost = 0.5 * cost;
    }
  }
  free(coeffs); free(df); free(dp); free(col_of_row); free(col_fixed);
  free(row_v); free(row_k); free(mask); free(Q); free(A); free(Ai);
  return ret;
}

int oracle_solve_linear_batch(int N, int D, int K, int r, int nd, int64_t B, const double* values,
                              const uint32_t* mask, const double* times, double* coeffs,
                              double* cost, int threads) {
  const int V = K + 1;
  int err = 0;
#ifdef _OPENMP
  base_init(); /* (before the parallel region: see base_ctor) */
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16) reduction(| : err)
#endif
  for (int64_t b = 0; b < B; ++b) {
    oracle_problem p = {N, D, K, r, nd, values + (size_t)b * V * nd * D, mask + (size_t)b * V,
                        times + (size_t)b * K};
    oracle_outputs o;
    memset(&o, 0, sizeof(o));
    o.coeffs = coeffs ? coeffs + (size_t)b * K * D * N : NULL;
    o.cost = cost ? cost + b : NULL;
    int rc = oracle_solve_linear(&p, &o);
    if (rc < 0) err |= 1;
  }
  (void)threads;
  return err ? ORACLE_ERR_ARG : ORACLE_OK;
}

/* ------------------------------------------------------------------------ */
/* Trajectory::evaluateRange (src/trajectory.cpp:68-128)                    */
/* ------------------------------------------------------------------------ */
int64_t oracle_evaluate_range(int N, int D, int K, const double* coeffs, const double* times,
                              double t_start, double t_end, double dt, int derivative,
                              int64_t max_samples, double* out, double* sample_times) {
  double accumulated_time = 0.0;
  int i = 0;
  for (i = 0; i < K; ++i) {
    accumulated_time += times[i];
    if (accumulated_time > t_start) break;
  }
  if (t_start > accumulated_time) return 0; /* LOG(ERROR) "Start time out of range" */
  if (i >= K) i = K - 1; /* loop ran out exactly at t_start == total (reference indexes [i]) */
  accumulated_time -= times[i];
  double time_in_segment = t_start - accumulated_time;
  int64_t n = 0;
  while (accumulated_time < t_end) {
    if (time_in_segment > times[i]) {
      time_in_segment = time_in_segment - times[i];
      i++;
      if (i >= K) break;
      continue;
    }
    if (n < max_samples) {
      for (int d = 0; d < D; ++d)
        out[n * D + d] = oracle_poly_evaluate(N, coeffs + ((size_t)i * D + d) * N, time_in_segment, derivative);
      if (sample_times) sample_times[n] = accumulated_time;
    }
    ++n;
    time_in_segment += dt;
    accumulated_time += dt;
  }
  return n;
}

/* ------------------------------------------------------------------------ */
/* Cost of fixed vertex derivatives at candidate times (config 5 CPU side)  */
/* ------------------------------------------------------------------------ */
/* Segment i's share of J_d = sum_dims x^T H(T) x, x = [d_i; d_{i+1}] (2h derivatives), with
 * H = A^-T Q A^-1 formed as updateSegmentTimes (lin_impl:276-295) + constructR (:298-326) do. */
static double segment_cost(int N, int D, int r, int nd, double T, const double* x, int i) {
  const int h = N / 2;
  double A[ORACLE_KMAXN * ORACLE_KMAXN], Ai[ORACLE_KMAXN * ORACLE_KMAXN], Q[ORACLE_KMAXN * ORACLE_KMAXN];
  double T1[ORACLE_KMAXN * ORACLE_KMAXN], H[ORACLE_KMAXN * ORACLE_KMAXN];
  oracle_setup_mapping_matrix(N, T, A);
  oracle_invert_mapping_matrix(N, A, Ai);
  oracle_quadratic_cost_jacobian(N, r, T, Q);
  for (int p = 0; p < N; ++p)
    for (int q = 0; q < N; ++q) {
      double s = 0.0;
      for (int k = 0; k < N; ++k) s += Q[p * N + k] * Ai[k * N + q];
      T1[p * N + q] = s;
    }
  for (int p = 0; p < N; ++p)
    for (int q = 0; q < N; ++q) {
      double s = 0.0;
      for (int k = 0; k < N; ++k) s += Ai[k * N + p] * T1[k * N + q];
      H[p * N + q] = s;
    }
  double cost = 0.0;
  for (int d = 0; d < D; ++d) {
    double xs[ORACLE_KMAXN];
    for (int k = 0; k < h; ++k) {
      xs[k] = x[((size_t)i * nd + k) * D + d];
      xs[h + k] = x[((size_t)(i + 1) * nd + k) * D + d];
    }
    for (int p = 0; p < N; ++p) {
      double s = 0.0;
      for (int q = 0; q < N; ++q) s += H[p * N + q] * xs[q];
      cost += xs[p] * s;
    }
  }
  return cost;
}

int oracle_cost_at_times_batch(int N, int D, int K, int r, int nd, int64_t B, const double* xfull,
                               const double* times, int C, const double* scales, double* J,
                               int threads) {
  if (N < 2 || N > ORACLE_KMAXN || (N % 2) || K < 1 || D < 1 || C < 1 || nd < N / 2) return ORACLE_ERR_ARG;
  const int V = K + 1;
#ifdef _OPENMP
  base_init(); /* (before the parallel region: see base_ctor) */
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t b = 0; b < B; ++b) {
    const double* x = xfull + (size_t)b * V * nd * D;
    for (int c = 0; c < C; ++c) {
      double cost = 0.0;
      for (int i = 0; i < K; ++i)
        cost += segment_cost(N, D, r, nd, times[(size_t)b * K + i] * scales[(size_t)c * K + i], x, i);
      J[(size_t)b * C + c] = cost;
    }
  }
  (void)threads;
  return ORACLE_OK;
}

/* getCostAndGradientTime's J_d gradient (polynomial_optimization_nonlinear_impl.h:2172-2229):
 * for each segment n, updateSegmentTimes with T_n -+ increment_time (both 0.1 when T_n <= 0.1,
 * :2182, :2201), getCostAndGradientDerivative at each, central difference.  The full J_d sums are
 * recomputed as the reference does.  increment_time == 0 asks for the exact derivative: the limit
 * of the same central difference, taken by Richardson extrapolation over steps 2e-2 T_n / 2^k on
 * segment n's share (the other segments' shares cancel exactly in the difference). */
int oracle_cost_time_jacobian_batch(int N, int D, int K, int r, int nd, int64_t B, const double* xfull,
                                    const double* times, int C, const double* scales, double increment_time,
                                    double* J, double* G, int threads) {
  if (N < 2 || N > ORACLE_KMAXN || (N % 2) || K < 1 || D < 1 || C < 1 || nd < N / 2 || K > 256 ||
      !(increment_time >= 0.0))
    return ORACLE_ERR_ARG;
  const int V = K + 1;
#ifdef _OPENMP
  base_init(); /* (before the parallel region: see base_ctor) */
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t b = 0; b < B; ++b) {
    const double* x = xfull + (size_t)b * V * nd * D;
    double Tc[256], share[256];
    for (int c = 0; c < C; ++c) {
      double tot = 0.0;
      for (int i = 0; i < K; ++i) {
        Tc[i] = times[(size_t)b * K + i] * scales[(size_t)c * K + i];
        share[i] = segment_cost(N, D, r, nd, Tc[i], x, i);
        tot += share[i];
      }
      J[(size_t)b * C + c] = tot;
      if (!G) continue;
      for (int n = 0; n < K; ++n) {
        double g;
        if (increment_time > 0.0) {
          const double dt = increment_time;
          const double tm = Tc[n] <= 0.1 ? 0.1 : Tc[n] - dt, tp = Tc[n] <= 0.1 ? 0.1 : Tc[n] + dt;
          double jm = 0.0, jp = 0.0;
          for (int i = 0; i < K; ++i) {
            jm += i == n ? segment_cost(N, D, r, nd, tm, x, i) : share[i];
            jp += i == n ? segment_cost(N, D, r, nd, tp, x, i) : share[i];
          }
          g = (jp - jm) / (2.0 * dt);
        } else {
          double R[4][4];
          double hs = 2e-2 * Tc[n];
          for (int k = 0; k < 4; ++k, hs *= 0.5)
            R[k][0] = (segment_cost(N, D, r, nd, Tc[n] + hs, x, n) - segment_cost(N, D, r, nd, Tc[n] - hs, x, n)) /
                      (2.0 * hs);
          for (int j = 1; j < 4; ++j) {
            const double f = pow(4.0, j);
            for (int k = j; k < 4; ++k) R[k][j] = (f * R[k][j - 1] - R[k - 1][j - 1]) / (f - 1.0);
          }
          g = R[3][3];
        }
        G[((size_t)b * C + c) * K + n] = g;
      }
    }
  }
  (void)threads;
  return ORACLE_OK;
}
