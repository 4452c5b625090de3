// Single-problem latency of the C++ drop-in (BASELINE config 1 / the reference's only benchmark,
// src/polynomial_timing_evaluation.cpp:93-128): PolynomialOptimization<10>(3) + setupFromVertices +
// solveLinear, timed over the same span as the reference's timer, against the oracle restatement
// of the reference algorithm on one core (the CPU-baseline column; test infrastructure).
// Problems: createRandomVerticesPath(3, K, 5.0, SNAP, seed) + estimateSegmentTimes(2, 2, 6.5) via
// the library's bit-exact generator.  Host only: kAuto runs single problems on the host solver.
// Build + run: see scripts/latency_cpp.sh.
#include <chrono>
#include <cstdio>
#include <vector>

#include "mav_trajectory_generation/polynomial_optimization_linear.h"
extern "C" {
#include "mtg_oracle.h"
}

namespace mtg = mav_trajectory_generation;

int main() {
  const int N = 10, D = 3, r = 4, h = N / 2;
  for (int K : {2, 10, 50, 100}) {
    const int V = K + 1;
    std::vector<double> vals((size_t)V * h * D), times(K);
    std::vector<uint8_t> mask(V);
    mtg_host_random_vertices_path_batch(N, D, K, 5.0, 4, 1, 1, 2.0, 2.0, 6.5, vals.data(), mask.data(), times.data(), 1);
    mtg::Vertex::Vector vertices;
    for (int v = 0; v < V; ++v) {
      mtg::Vertex vx(D);
      for (int k = 0; k < h; ++k)
        if ((mask[v] >> k) & 1) {
          mtg::VectorXd c(D);
          for (int d = 0; d < D; ++d) c[d] = vals[((size_t)v * h + k) * D + d];
          vx.addConstraint(k, c);
        }
      vertices.push_back(vx);
    }
    const int reps = K <= 10 ? 20000 : K <= 50 ? 2000 : 300;
    double sink = 0.0;  // (the timed span is the reference's: ctor + setupFromVertices + solveLinear)
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) {
      mtg::PolynomialOptimization<10> opt(D);
      opt.setupFromVertices(vertices, times, r);
      opt.solveLinear();
    }
    auto t1 = std::chrono::steady_clock::now();
    const double drop_in_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
    std::vector<uint32_t> m32(mask.begin(), mask.end());
    std::vector<double> coeffs((size_t)K * D * N), cost(1);
    const int oreps = K <= 10 ? 20000 : K <= 50 ? 500 : 50;
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < oreps; ++i) {
      oracle_solve_linear_batch(N, D, K, r, h, 1, vals.data(), m32.data(), times.data(), coeffs.data(), cost.data(), 1);
      sink += cost[0];
    }
    t1 = std::chrono::steady_clock::now();
    const double oracle_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / oreps;
    std::printf("{\"K\": %d, \"drop_in_host_us\": %.2f, \"oracle_1core_us\": %.2f, \"reps\": %d, \"sink\": %.3g}\n", K,
                drop_in_us, oracle_us, reps, sink);
  }
  return 0;
}
