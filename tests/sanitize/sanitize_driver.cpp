// Host-only ASan/UBSan driver (tests/test_sanitizers.py): the library's host code
// (csrc/mtg_host.cpp: generators, segment-time estimate; csrc/mtg_host_solve.cpp: the host solve
// path and the host matrices; csrc/mtg_host_extrema.cpp: the host min/max magnitude) and the oracle's C restatement, compiled with -fsanitize and run on
// small problems of every N, odd and even K, mixed masks, K = 1, and the rejected shapes.  Any
// sanitizer report aborts the run (halt_on_error); the exit code is the number of failed checks.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "mtg.h"
extern "C" {
#include "mtg_oracle.h"
}

static int failures = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "check failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

static void solve_case(int N, int D, int K, int r, int B, unsigned seed, bool mixed) {
  const int h = N / 2, V = K + 1;
  std::vector<double> vals((size_t)B * V * h * D), times((size_t)B * K);
  std::vector<uint8_t> mask((size_t)B * V);
  const int maxd = h - 1 < 4 ? h - 1 : 4;
  CHECK(mtg_host_random_vertices_path_batch(N, D, K, 5.0, maxd, seed, B, 2.0, 2.0, 6.5, vals.data(), mask.data(),
                                            times.data(), 2) == MTG_OK);
  if (mixed)  // extra fixed derivatives at interior vertices, different per trajectory
    for (int b = 0; b < B; ++b)
      for (int v = 1; v < K; ++v) mask[(size_t)b * V + v] |= (uint8_t)((b + v) & ((1 << h) - 2));
  std::vector<double> coeffs((size_t)B * K * D * N), freev((size_t)B * D * V * h), cost(B);
  std::vector<int32_t> nfree(B), status(B);
  CHECK(mtg_host_solve_linear_batch(N, D, K, r, B, vals.data(), mask.data(), times.data(), coeffs.data(),
                                    freev.data(), nfree.data(), cost.data(), status.data(), 2) == MTG_OK);
  for (int b = 0; b < B; ++b) CHECK((status[b] & MTG_TRAJ_ERROR_MASK) == 0);
  for (double c : coeffs) CHECK(std::isfinite(c));
  // the oracle restatement on the same problems
  std::vector<uint32_t> m32(mask.begin(), mask.end());
  std::vector<double> ocoef((size_t)B * K * D * N), ocost(B);
  CHECK(oracle_solve_linear_batch(N, D, K, r, h, B, vals.data(), m32.data(), times.data(), ocoef.data(),
                                  ocost.data(), 2) == 0);
  double err = 0.0;
  for (size_t i = 0; i < coeffs.size(); ++i) err = std::fmax(err, std::fabs(coeffs[i] - ocoef[i]));
  CHECK(std::isfinite(err));
  // evaluateRange of the first trajectory
  std::vector<double> out(4096 * D), st(4096);
  const int64_t n = oracle_evaluate_range(N, D, K, coeffs.data(), times.data(), 0.0, 1e9, 0.05, 1, 4096,
                                          out.data(), st.data());
  CHECK(n > 0);
  // coefficients from the solved vertex values and the per-segment matrices
  std::vector<double> full((size_t)B * V * h * D, 0.0), c2((size_t)B * K * D * N);
  for (int b = 0; b < B; ++b)
    for (int v = 0; v < V; ++v)
      for (int k = 0; k < h; ++k)
        for (int d = 0; d < D; ++d) {
          const size_t i = (((size_t)b * V + v) * h + k) * D + d;
          full[i] = vals[i];
        }
  CHECK(mtg_host_coefficients_from_vertices_batch(N, D, K, B, full.data(), times.data(), c2.data(), 2) == MTG_OK);
  std::vector<double> A(N * N), Ai(N * N), Q(N * N), H(N * N);
  CHECK(mtg_host_segment_matrices(N, r, times[0], A.data(), Ai.data(), Q.data(), H.data()) == MTG_OK);
  // min / max magnitude of every derivative the host path accepts, all and one dimension
  std::vector<mtg_extremum> mn(B), mx(B);
  for (int k = 0; k <= N - 2; ++k) {
    CHECK(mtg_host_min_max_magnitude_batch(N, D, K, B, coeffs.data(), times.data(), k, 0, mn.data(), mx.data(), 2) ==
          MTG_OK);
    CHECK(mtg_host_min_max_magnitude_batch(N, D, K, B, coeffs.data(), times.data(), k, 1u, mn.data(), nullptr, 1) ==
          MTG_OK);
    for (int b = 0; b < B; ++b) CHECK(mx[b].segment >= 0 && mx[b].segment < K && std::isfinite(mx[b].value));
  }
  std::vector<double> oA(N * N), oAi(N * N), oQ(N * N);
  oracle_setup_mapping_matrix(N, times[0], oA.data());
  oracle_invert_mapping_matrix(N, oA.data(), oAi.data());
  oracle_quadratic_cost_jacobian(N, r, times[0], oQ.data());
}

int main() {
  for (int N = 4; N <= 12; N += 2)  // (N = 2: the generators need max_derivative >= 1)
    for (int K : {1, 2, 5, 8}) {
      const int r = N / 2 - 1;
      solve_case(N, 3, K, r, 5, 100 + N + K, false);
      if (N >= 4 && K > 1) solve_case(N, 2, K, r > 0 ? r - 1 : 0, 4, 200 + N + K, true);
    }
  solve_case(10, 1, 20, 4, 3, 7, false);
  // rejected shapes return an error, never touch memory
  double dummy = 0.0;
  uint8_t m = 0;
  CHECK(mtg_host_solve_linear_batch(11, 3, 10, 4, 1, &dummy, &m, &dummy, &dummy, nullptr, nullptr, nullptr, nullptr,
                                    1) != MTG_OK);
  CHECK(mtg_host_solve_linear_batch(10, 3, 10, 5, 1, &dummy, &m, &dummy, &dummy, nullptr, nullptr, nullptr, nullptr,
                                    1) != MTG_OK);
  std::vector<double> pos(3 * 4);
  for (size_t i = 0; i < pos.size(); ++i) pos[i] = (double)i;
  std::vector<double> t(3);
  CHECK(mtg_host_estimate_segment_times(4, 3, pos.data(), 2.0, 2.0, 6.5, t.data()) == MTG_OK);
  std::printf("sanitize driver: %d failed checks\n", failures);
  return failures ? 1 : 0;
}
