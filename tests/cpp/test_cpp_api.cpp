// C++ API test (include/mtg/trajectory_generation.hpp over libmtg.so), written the way the
// reference's own tests use PolynomialOptimization (test/test_polynomial_optimization.cpp).
// Needs a HIP device: run by tests/test_cpp_api.py under -m gpu; compiled (not run) on CPU.
// Exit status 0 = all checks passed.
#define MTG_CPP_THROW 1
#include "mtg/trajectory_generation.hpp"

#include <cmath>
#include <cstdio>
#include <vector>

using namespace mtg;

static int g_fail = 0;
#define EXPECT(cond, ...)                                   \
  do {                                                      \
    if (!(cond)) {                                          \
      ++g_fail;                                             \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                    \
      std::fprintf(stderr, "\n");                           \
    }                                                       \
  } while (0)

static double maxabs(const std::vector<double>& v) {
  double m = 0;
  for (double x : v) m = std::fmax(m, std::fabs(x));
  return m;
}

// checkPath (test_polynomial_optimization.cpp:73-131), tolerance relative to the derivative's scale
// (the reference's absolute 1e-6 does not hold on millisecond segments; DESIGN.md "Parity")
template <int N>
static void checkPath(const Vertex::Vector& vertices, const Segment::Vector& segments, double tol) {
  EXPECT(segments.size() + 1 == vertices.size(), "segment count");
  for (size_t i = 0; i < segments.size(); ++i) {
    const Segment& s = segments[i];
    for (int end = 0; end < 2; ++end) {
      const Vertex& vx = vertices[i + end];
      const double t = end ? s.getTime() : 0.0;
      for (auto it = vx.cBegin(); it != vx.cEnd(); ++it) {
        if (it->first >= N / 2) continue;
        const auto actual = s.evaluate(t, it->first);
        const double scale = std::fmax(1.0, maxabs(it->second));
        for (int d = 0; d < s.D(); ++d)
          EXPECT(std::fabs(actual[d] - it->second[d]) <= tol * scale, "fixed constraint seg %zu end %d der %d", i, end,
                 it->first);
      }
    }
    if (i > 0) {
      const Segment& p = segments[i - 1];
      for (int der = 0; der < N / 2; ++der) {
        const auto a = p.evaluate(p.getTime(), der), b = s.evaluate(0.0, der);
        const double scale = std::fmax(1.0, std::fmax(maxabs(a), maxabs(b)));
        for (int d = 0; d < s.D(); ++d)
          EXPECT(std::fabs(a[d] - b[d]) <= tol * scale, "continuity at vertex %zu der %d", i, der);
      }
    }
  }
}

// test_polynomial_optimization.cpp:700-744 (MATLAB coefficients)
static void test_two_vertices_setup() {
  Vertex::Vector vertices;
  Vertex start(1), end(1);
  start.makeStartOrEnd(0.0, derivative_order::SNAP);
  end.makeStartOrEnd(5.0, derivative_order::SNAP);
  vertices.push_back(start);
  vertices.push_back(end);
  PolynomialOptimization<10> opt(1);
  opt.setupFromVertices(vertices, {5.0}, derivative_order::SNAP);
  opt.solveLinear();
  Segment::Vector segments;
  opt.getSegments(&segments);
  const double matlab[10] = {-0.000000000000004, 0.000000000000004, -0.000000000000006, 0.000000000000003,
                             -0.000000000000001, 0.201600000000015, -0.134400000000012, 0.034560000000004,
                             -0.004032000000000, 0.000179200000000};
  const auto& c = segments[0][0].getCoefficients();
  for (int j = 0; j < 10; ++j) EXPECT(std::fabs(c[j] - matlab[j]) <= 1e-13, "2_vertices_setup c[%d]", j);
  EXPECT(opt.getNumberFreeConstraints() == 0, "n_free");
}

// createRandomVertices + estimateSegmentTimes through the product's host generator, then the
// single-trajectory API; checkPath and cost consistency (PathPlanning tests :280-420)
template <int N>
static void test_random_paths(int D, int K, int max_derivative, int r, int seeds) {
  const int h = N / 2, V = K + 1;
  std::vector<double> pmin(D, -10.0), pmax(D, 10.0);
  for (int seed = 0; seed < seeds; ++seed) {
    std::vector<double> values((size_t)V * h * D);
    std::vector<uint8_t> mask(V);
    std::vector<double> times(K);
    EXPECT(mtg_host_random_vertices_batch(N, D, K, max_derivative, pmin.data(), pmax.data(), 1000 + seed, 1, 3.0,
                                          5.0, 6.5, values.data(), mask.data(), times.data(), 1) == MTG_OK,
           "generator");
    Vertex::Vector vertices;
    for (int v = 0; v < V; ++v) {
      Vertex vx(D);
      for (int k = 0; k < h; ++k)
        if ((mask[v] >> k) & 1u) {
          std::vector<double> c(D);
          for (int d = 0; d < D; ++d) c[d] = values[((size_t)v * h + k) * D + d];
          vx.addConstraint(k, c);
        }
      vertices.push_back(vx);
    }
    PolynomialOptimization<N> opt(D);
    opt.setupFromVertices(vertices, times, r);
    opt.solveLinear();
    Segment::Vector segments;
    opt.getSegments(&segments);
    checkPath<N>(vertices, segments, 1e-8);
    EXPECT(std::isfinite(opt.computeCost()) && opt.computeCost() >= 0.0, "cost");
    EXPECT(opt.getNumberAllConstraints() == (size_t)V * h, "all constraints");

    // the batched entry point gives the same coefficients
    BatchPolynomialOptimization<N> batch(D, K, r);
    std::vector<double> coeffs((size_t)K * D * N);
    double cost = 0.0;
    batch.solve(1, values.data(), mask.data(), times.data(), coeffs.data(), &cost);
    for (int i = 0; i < K; ++i)
      for (int d = 0; d < D; ++d) {
        const auto& c = segments[i][d].getCoefficients();
        for (int j = 0; j < N; ++j) EXPECT(c[j] == coeffs[((size_t)i * D + d) * N + j], "batch vs single");
      }
    EXPECT(cost == opt.computeCost(), "batch cost");
  }
}

// ConstraintPacking (test_polynomial_optimization.cpp:600-698): counts and (vertex, derivative) order
static void test_constraint_packing() {
  const int K = 5, D = 3;
  Vertex::Vector vertices;
  for (int v = 0; v <= K; ++v) {
    Vertex vx(D);
    if (v == 0 || v == K)
      vx.makeStartOrEnd(std::vector<double>{1.0 * v, 2.0, 3.0}, derivative_order::JERK);
    else
      vx.addConstraint(derivative_order::POSITION, std::vector<double>{1.0 * v, -1.0 * v, 0.5 * v});
    vertices.push_back(vx);
  }
  PolynomialOptimization<10> opt(D);
  opt.setupFromVertices(vertices, std::vector<double>(K, 1.5), derivative_order::SNAP);
  opt.solveLinear();
  // ends: derivatives 0..3 fixed (4 each), interior: position (1 each)
  EXPECT(opt.getNumberFixedConstraints() == 2 * 4 + (K - 1), "n_fixed %zu", opt.getNumberFixedConstraints());
  EXPECT(opt.getNumberFreeConstraints() == 2 * 1 + (K - 1) * 4, "n_free %zu", opt.getNumberFreeConstraints());
  std::vector<std::vector<double>> fc;
  opt.getFreeConstraints(&fc);
  EXPECT(fc.size() == (size_t)D && fc[0].size() == opt.getNumberFreeConstraints(), "free shape");
  // the first free value is vertex 0's snap; evaluating the start segment's 4th derivative must match it
  Segment::Vector segments;
  opt.getSegments(&segments);
  for (int d = 0; d < D; ++d)
    EXPECT(std::fabs(segments[0].evaluate(0.0, derivative_order::SNAP)[d] - fc[d][0]) <=
               1e-9 * std::fmax(1.0, std::fabs(fc[d][0])),
           "free snap at vertex 0, dim %d", d);
}

// evaluateRange: count, times and values against per-sample Trajectory::evaluate
static void test_evaluate_range() {
  Vertex::Vector vertices;
  for (int v = 0; v <= 3; ++v) {
    Vertex vx(2);
    if (v == 0 || v == 3)
      vx.makeStartOrEnd(std::vector<double>{1.0 * v, -2.0 * v}, derivative_order::SNAP);
    else
      vx.addConstraint(derivative_order::POSITION, std::vector<double>{1.0 * v + 0.3, 0.7 * v});
    vertices.push_back(vx);
  }
  PolynomialOptimization<10> opt(2);
  opt.setupFromVertices(vertices, {1.0, 2.0, 1.5});
  opt.solveLinear();
  Trajectory traj;
  opt.getTrajectory(&traj);
  std::vector<std::vector<double>> samples;
  std::vector<double> st;
  traj.evaluateRange(0.0, traj.getMaxTime(), 0.01, derivative_order::POSITION, &samples, &st);
  EXPECT(samples.size() == st.size() && samples.size() >= 449 && samples.size() <= 451, "samples %zu", samples.size());
  // computeMinMaxMagnitude (trajectory.cpp:181-218) against the sampled speed
  Trajectory::Extremum vmin, vmax;
  EXPECT(traj.computeMinMaxMagnitude(derivative_order::VELOCITY, {0, 1}, &vmin, &vmax), "min/max magnitude");
  std::vector<std::vector<double>> vel;
  traj.evaluateRange(0.0, traj.getMaxTime(), 0.001, derivative_order::VELOCITY, &vel);
  double smax = 0.0;
  for (const auto& v : vel) smax = std::fmax(smax, std::sqrt(v[0] * v[0] + v[1] * v[1]));
  EXPECT(vmax.value >= smax * (1 - 1e-12) && vmax.value <= smax * (1 + 1e-4), "max speed %g vs sampled %g", vmax.value,
         smax);
  EXPECT(vmin.value <= 1e-9 && vmax.segment_idx >= 0 && vmax.segment_idx < 3, "min speed %g (rest at the ends)",
         vmin.value);
  for (size_t s = 0; s < samples.size(); s += 37) {
    const auto e = traj.evaluate(st[s], derivative_order::POSITION);
    for (int d = 0; d < 2; ++d)
      EXPECT(std::fabs(e[d] - samples[s][d]) <= 1e-12 * std::fmax(1.0, std::fabs(e[d])), "sample %zu", s);
  }
}

// error behaviour: CHECKs of setupFromVertices (lin_impl:50-55, :66-67) as mtg::Error here
static void test_errors() {
  Vertex::Vector vertices(2, Vertex(1));
  vertices[0].makeStartOrEnd(0.0, 4);
  vertices[1].makeStartOrEnd(1.0, 4);
  PolynomialOptimization<10> opt(1);
  bool threw = false;
  try {
    opt.setupFromVertices(vertices, {1.0}, 5);
  } catch (const Error& e) {
    threw = e.code == MTG_ERR_BAD_DERIVATIVE;
  }
  EXPECT(threw, "derivative 5 for N=10 must fail");
  threw = false;
  try {
    opt.setupFromVertices(vertices, {1.0, 2.0});
  } catch (const Error& e) {
    threw = e.code == MTG_ERR_SIZE_MISMATCH;
  }
  EXPECT(threw, "size mismatch must fail");
  threw = false;
  try {
    opt.setupFromVertices(vertices, {-1.0});
  } catch (const Error&) {
    threw = true;
  }
  EXPECT(threw, "negative time must fail");
}

// setFreeConstraints round trip and computeInitialSolutionWithoutPositionConstraints (nl_impl:116-187)
static void test_free_constraints_and_reparametrisation() {
  const int K = 6, D = 3, N = 10;
  Vertex::Vector vertices;
  for (int v = 0; v <= K; ++v) {
    Vertex vx(D);
    if (v == 0 || v == K)
      vx.makeStartOrEnd(std::vector<double>{1.0 * v, 2.0 - v, 0.5}, derivative_order::SNAP);
    else
      vx.addConstraint(derivative_order::POSITION, std::vector<double>{1.0 * v + 0.2 * (v % 2), -0.7 * v, 0.3 * v * v});
    vertices.push_back(vx);
  }
  std::vector<double> times{1.1, 0.8, 1.7, 2.2, 0.9, 1.3};
  PolynomialOptimization<N> opt(D);
  opt.setupFromVertices(vertices, times, derivative_order::SNAP);
  opt.solveLinear();
  Segment::Vector s0;
  opt.getSegments(&s0);
  const double cost0 = opt.computeCost();
  std::vector<std::vector<double>> fc, fx;
  opt.getFreeConstraints(&fc);
  opt.getFixedConstraints(&fx);
  EXPECT(fx.size() == (size_t)D && fx[0].size() == opt.getNumberFixedConstraints(), "fixed shape");
  opt.setFreeConstraints(fc);  // same values: same polynomials and cost
  Segment::Vector s1;
  opt.getSegments(&s1);
  for (int i = 0; i < K; ++i)
    for (int d = 0; d < D; ++d)
      for (int j = 0; j < N; ++j) {
        const double a = s0[i][d].getCoefficients()[j], b = s1[i][d].getCoefficients()[j];
        EXPECT(std::fabs(a - b) <= 1e-12 * std::fmax(1.0, std::fabs(a)), "setFreeConstraints coefficient");
      }
  EXPECT(std::fabs(opt.computeCost() - cost0) <= 1e-9 * cost0, "cost after setFreeConstraints");
  const size_t nf0 = opt.getNumberFreeConstraints();
  computeInitialSolutionWithoutPositionConstraints(&opt);
  EXPECT(opt.getNumberFreeConstraints() == nf0 + (K - 1), "n_free after releasing positions %zu",
         opt.getNumberFreeConstraints());
  Segment::Vector s2;
  opt.getSegments(&s2);
  for (int i = 0; i < K; ++i)
    for (int d = 0; d < D; ++d) {
      double sc = 0.0, err = 0.0, tp = 1.0;
      for (int j = 0; j < N; ++j, tp *= times[i]) {
        sc = std::fmax(sc, std::fabs(s0[i][d].getCoefficients()[j]) * tp);
        err = std::fmax(err, std::fabs(s0[i][d].getCoefficients()[j] - s2[i][d].getCoefficients()[j]) * tp);
      }
      EXPECT(err <= 1e-9 * sc, "re-parametrised trajectory differs: seg %d dim %d (%g)", i, d, err / sc);
    }
  EXPECT(std::fabs(opt.computeCost() - cost0) <= 1e-8 * cost0, "cost after re-parametrisation");
}

int main() {
  test_free_constraints_and_reparametrisation();
  test_two_vertices_setup();
  test_random_paths<10>(3, 10, 4, 4, 20);
  test_random_paths<8>(2, 6, 3, 2, 10);
  test_random_paths<12>(3, 20, 4, 3, 5);
  test_constraint_packing();
  test_evaluate_range();
  test_errors();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("test_cpp_api: all checks passed\n");
  return 0;
}
