// mtg_host.cpp -- host utilities of libmav_trajectory_generation.so (no GPU): the reference's
// synthetic problem generators, bit-exact with libstdc++ <random> because
// they use it, packed straight into the ABI layout of include/mtg.h.
//
//   createRandomVertices       src/vertex.cpp:27-79
//   createRandomVerticesPath   src/polynomial_timing_evaluation.cpp:34-91
//   estimateSegmentTimes       src/vertex.cpp:162-178
//
// Eigen's VectorXd::norm()/normalized() are reproduced with Eigen's own
// reduction order for SSE2 packets of two doubles (Eigen/src/Core/Redux.h), so
// the generated positions and times are bit-identical to what the reference
// binary would produce on x86-64.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "mtg.h"
#include "mtg_host_threads.h"

namespace {

double eigen_squared_norm(const double* x, int n) {
  if (n <= 0) return 0.0;
  const int aligned2 = (n / 4) * 4, aligned = (n / 2) * 2;
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

// One generated vertex list in "reference" form: per vertex the set of
// constrained derivatives (bit k) and their values [derivative][D].
struct Gen {
  int V, D, nd;
  std::vector<double> val;    // [V][nd][D]
  std::vector<uint32_t> bits; // [V]
  Gen(int V_, int D_, int nd_) : V(V_), D(D_), nd(nd_), val((size_t)V_ * nd_ * D_, 0.0), bits(V_, 0u) {}
  void set(int v, int k, const double* x) {
    for (int d = 0; d < D; ++d) val[((size_t)v * nd + k) * D + d] = x[d];
    bits[v] |= 1u << k;
  }
  // Vertex::makeStartOrEnd (src/vertex.cpp:106-112)
  void start_or_end(int v, const double* pos, int up_to) {
    set(v, 0, pos);
    std::vector<double> z(D, 0.0);
    for (int k = 1; k <= up_to; ++k) set(v, k, z.data());
  }
};

void gen_random_vertices(int max_derivative, int K, int D, const double* pos_min, const double* pos_max,
                         uint32_t seed, Gen* g) {
  std::mt19937 generator(seed);
  std::vector<std::uniform_real_distribution<double>> dist(D);
  for (int i = 0; i < D; ++i) dist[i] = std::uniform_real_distribution<double>(pos_min[i], pos_max[i]);
  const double min_distance = 0.2;
  const int V = K + 1;
  std::vector<double> last(D), pos(D), diff(D);
  for (int i = 0; i < D; ++i) last[i] = dist[i](generator);
  g->start_or_end(0, last.data(), max_derivative);
  for (int i = 1; i < V; ++i) {
    for (;;) {
      for (int d = 0; d < D; ++d) pos[d] = dist[d](generator);
      for (int d = 0; d < D; ++d) diff[d] = pos[d] - last[d];
      if (std::sqrt(eigen_squared_norm(diff.data(), D)) > min_distance) break;
    }
    g->set(i, 0, pos.data());
    last = pos;
  }
  g->start_or_end(V - 1, last.data(), max_derivative);
}

void gen_random_vertices_path(int D, int K, double average_distance, int max_derivative, uint32_t seed,
                              Gen* g) {
  std::mt19937 generator(seed);
  std::vector<std::uniform_real_distribution<double>> dist(D);
  std::uniform_real_distribution<double> random_distance(0, 2 * average_distance);
  for (int i = 0; i < D; ++i) dist[i] = std::uniform_real_distribution<double>(-1, 1);
  const double min_distance = 0.2;
  const int V = K + 1;
  std::vector<double> last(D), ps(D), vtx(D);
  for (int i = 0; i < D; ++i) last[i] = dist[i](generator);
  g->start_or_end(0, last.data(), max_derivative);
  for (int i = 1; i < V; ++i) {
    for (;;) {
      for (int d = 0; d < D; ++d) ps[d] = dist[d](generator);
      if (std::sqrt(eigen_squared_norm(ps.data(), D)) > min_distance) break;
    }
    // position_sample.normalized() * random_distance(generator)  (:78)
    const double z = eigen_squared_norm(ps.data(), D);
    const double s = std::sqrt(z);
    const double r = random_distance(generator);
    for (int d = 0; d < D; ++d) ps[d] = (z > 0.0 ? ps[d] / s : ps[d]) * r;
    for (int d = 0; d < D; ++d) vtx[d] = ps[d] + last[d];
    g->set(i, 0, vtx.data());
    last = ps;  // the reference keeps the offset, not the position (:86)
  }
  g->start_or_end(V - 1, last.data(), max_derivative);  // overwrites the last position (:88)
}

void estimate_times(const Gen& g, double v_max, double a_max, double magic, double* times) {
  const int D = g.D;
  std::vector<double> diff(D);
  for (int i = 0; i + 1 < g.V; ++i) {
    const double* s = &g.val[((size_t)i * g.nd) * D];
    const double* e = &g.val[((size_t)(i + 1) * g.nd) * D];
    for (int d = 0; d < D; ++d) diff[d] = e[d] - s[d];
    const double distance = std::sqrt(eigen_squared_norm(diff.data(), D));
    times[i] = distance / v_max * 2 * (1.0 + magic * v_max / a_max * std::exp(-distance / v_max * 2));
  }
}

// Pack one generated vertex list into values [V][h][D] / mask [V] (uint8).
void pack(const Gen& g, int N, double* values, uint8_t* mask) {
  const int h = N / 2, D = g.D;
  std::memset(values, 0, sizeof(double) * (size_t)g.V * h * D);
  for (int v = 0; v < g.V; ++v) {
    uint32_t b = g.bits[v];
    uint8_t m = (uint8_t)(b & 0x7fu);
    if (b >> 7) m |= 0x80u;  // orders >= 7 collapse into bit 7 (dropped by the solver anyway)
    mask[v] = m;
    for (int k = 0; k < h && k < g.nd; ++k)
      if ((b >> k) & 1u)
        for (int d = 0; d < D; ++d) values[((size_t)v * h + k) * D + d] = g.val[((size_t)v * g.nd + k) * D + d];
  }
}

template <typename F>
void parallel_for(int64_t n, int threads, F f) {
  int t = threads > 0 ? threads : mtg::usable_cpus();
  t = (int)std::min<int64_t>(t, std::max<int64_t>(1, n / 64));
  if (t <= 1) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> pool;
  for (int w = 0; w < t; ++w)
    pool.emplace_back([=, &f]() {
      for (int64_t i = w; i < n; i += t) f(i);
    });
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

int mtg_host_random_vertices_batch(int N, int D, int K, int max_derivative, const double* pos_min,
                                   const double* pos_max, uint32_t seed0, int64_t batch,
                                   double v_max, double a_max, double magic_fabian_constant,
                                   double* values, uint8_t* fixed_mask, double* times, int threads) {
  if (N < 2 || N > 12 || (N % 2) || D < 1 || K < 1 || batch < 0 || max_derivative <= 0 || !pos_min ||
      !pos_max || !values || !fixed_mask || !times)
    return MTG_ERR_INVALID_ARGUMENT;
  const int V = K + 1, h = N / 2;
  const int nd = std::max(max_derivative + 1, h);
  parallel_for(batch, threads, [&](int64_t b) {
    Gen g(V, D, nd);
    gen_random_vertices(max_derivative, K, D, pos_min, pos_max, seed0 + (uint32_t)b, &g);
    pack(g, N, values + (size_t)b * V * h * D, fixed_mask + (size_t)b * V);
    estimate_times(g, v_max, a_max, magic_fabian_constant, times + (size_t)b * K);
  });
  return MTG_OK;
}

int mtg_host_random_vertices_path_batch(int N, int D, int K, double average_distance,
                                        int max_derivative, uint32_t seed0, int64_t batch,
                                        double v_max, double a_max, double magic_fabian_constant,
                                        double* values, uint8_t* fixed_mask, double* times,
                                        int threads) {
  if (N < 2 || N > 12 || (N % 2) || D < 1 || K < 1 || batch < 0 || max_derivative <= 0 || !values ||
      !fixed_mask || !times)
    return MTG_ERR_INVALID_ARGUMENT;
  const int V = K + 1, h = N / 2;
  const int nd = std::max(max_derivative + 1, h);
  parallel_for(batch, threads, [&](int64_t b) {
    Gen g(V, D, nd);
    gen_random_vertices_path(D, K, average_distance, max_derivative, seed0 + (uint32_t)b, &g);
    pack(g, N, values + (size_t)b * V * h * D, fixed_mask + (size_t)b * V);
    estimate_times(g, v_max, a_max, magic_fabian_constant, times + (size_t)b * K);
  });
  return MTG_OK;
}

}  // extern "C"

extern "C" int mtg_host_estimate_segment_times(int n_vertices, int D, const double* positions, double v_max,
                                               double a_max, double magic_fabian_constant, double* times) {
  if (n_vertices < 1 || D < 1 || !positions || (n_vertices > 1 && !times)) return MTG_ERR_INVALID_ARGUMENT;
  Gen g(n_vertices, D, 1);
  for (int v = 0; v < n_vertices; ++v) g.set(v, 0, positions + (size_t)v * D);
  estimate_times(g, v_max, a_max, magic_fabian_constant, times);
  return MTG_OK;
}
