// ThreadSanitizer driver (tests/test_sanitizers.py): every multi-threaded host path, each one's
// FIRST call in a fresh process made with 8 threads -- the oracle's OpenMP solve (the race class of
// round 3: a table filled lazily inside the parallel region), the product's host solve, generators,
// host extrema and vertex maps (std::thread pools) -- then the same calls single-threaded, which
// must give bit-identical results.  Any TSan report fails the run (halt_on_error); the exit code is
// the number of failed checks.  argv[1] picks which path goes first ("oracle" or "host"), so that
// each of them is run as a fresh process's first threaded call.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mtg.h"
extern "C" {
#include "mtg_oracle.h"
}

static int failures = 0;
#define CHECK(c)                                                                    \
  do {                                                                              \
    if (!(c)) {                                                                     \
      std::fprintf(stderr, "check failed %s:%d: %s\n", __FILE__, __LINE__, #c);     \
      ++failures;                                                                   \
    }                                                                               \
  } while (0)

static const int N = 10, D = 3, K = 10, R = 4, H = N / 2, V = K + 1;
static const int B = 1024;  // >= 64 per worker, so every pool really runs 8 workers

struct Batch {
  std::vector<double> vals, times;
  std::vector<uint8_t> mask;
};

static Batch generate(int threads) {
  Batch b;
  b.vals.resize((size_t)B * V * H * D);
  b.times.resize((size_t)B * K);
  b.mask.resize((size_t)B * V);
  CHECK(mtg_host_random_vertices_path_batch(N, D, K, 5.0, 4, 11, B, 2.0, 2.0, 6.5, b.vals.data(), b.mask.data(),
                                            b.times.data(), threads) == MTG_OK);
  return b;
}

static std::vector<double> oracle_solve(const Batch& b, int threads) {
  std::vector<uint32_t> m32(b.mask.begin(), b.mask.end());
  std::vector<double> c((size_t)B * K * D * N), cost(B);
  CHECK(oracle_solve_linear_batch(N, D, K, R, H, B, b.vals.data(), m32.data(), b.times.data(), c.data(), cost.data(),
                                  threads) == 0);
  c.insert(c.end(), cost.begin(), cost.end());
  return c;
}

static std::vector<double> host_solve(const Batch& b, int threads) {
  std::vector<double> c((size_t)B * K * D * N), fr((size_t)B * D * V * H), cost(B);
  std::vector<int32_t> nf(B), st(B);
  CHECK(mtg_host_solve_linear_batch(N, D, K, R, B, b.vals.data(), b.mask.data(), b.times.data(), c.data(), fr.data(),
                                    nf.data(), cost.data(), st.data(), threads) == MTG_OK);
  for (int i = 0; i < B; ++i) CHECK(st[i] == 0);
  c.insert(c.end(), fr.begin(), fr.end());
  c.insert(c.end(), cost.begin(), cost.end());
  return c;
}

static std::vector<double> host_extrema(const std::vector<double>& coeffs, const Batch& b, int threads) {
  std::vector<mtg_extremum> mn(B), mx(B);
  CHECK(mtg_host_min_max_magnitude_batch(N, D, K, B, coeffs.data(), b.times.data(), 1, 0, mn.data(), mx.data(),
                                         threads) == MTG_OK);
  std::vector<double> o;
  for (int i = 0; i < B; ++i) o.insert(o.end(), {mn[i].value, mn[i].time, (double)mn[i].segment, mx[i].value,
                                                  mx[i].time, (double)mx[i].segment});
  return o;
}

static std::vector<double> host_vertex_map(const Batch& b, int threads) {
  std::vector<double> c((size_t)B * K * D * N);
  CHECK(mtg_host_coefficients_from_vertices_batch(N, D, K, B, b.vals.data(), b.times.data(), c.data(), threads) ==
        MTG_OK);
  return c;
}

static bool same(const std::vector<double>& a, const std::vector<double>& b) {
  return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(double)) == 0;
}

int main(int argc, char** argv) {
  const std::string first = argc > 1 ? argv[1] : "oracle";
  CHECK(mtg_host_default_threads() >= 1);
  std::vector<double> o8, h8;
  Batch g8;
  if (first == "oracle") {  // the oracle's first call is the threaded one (its tables not yet built)
    Batch g1 = generate(1);
    o8 = oracle_solve(g1, 8);
    g8 = generate(8);
    h8 = host_solve(g8, 8);
  } else {                  // the product's host paths first
    g8 = generate(8);
    h8 = host_solve(g8, 8);
    o8 = oracle_solve(g8, 8);
  }
  const std::vector<double> e8 = host_extrema(h8, g8, 8), v8 = host_vertex_map(g8, 8);
  const Batch g1 = generate(1);
  CHECK(g1.vals == g8.vals && g1.times == g8.times && g1.mask == g8.mask);
  CHECK(same(oracle_solve(g1, 1), o8));
  CHECK(same(host_solve(g1, 1), h8));
  CHECK(same(host_extrema(h8, g1, 1), e8));
  CHECK(same(host_vertex_map(g1, 1), v8));
  std::printf("tsan driver (%s first): %d failed checks\n", first.c_str(), failures);
  return failures ? 1 : 0;
}
