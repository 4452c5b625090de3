// C++ API test of the drop-in headers (include/mav_trajectory_generation/*.h, namespace
// mav_trajectory_generation) over libmav_trajectory_generation.so, written the way the reference's
// own tests use the API (test/test_polynomial_optimization.cpp).  Built by CMake (target
// test_cpp_api) or directly by tests/test_cpp_api.py.
//
//   test_cpp_api host          single problems on the library's host solver (no GPU needed)
//   test_cpp_api device        single problems through the GPU (ExecutionPolicy::kDevice) and the
//                              batched API; needs a HIP device
//   test_cpp_api dump <file>   write getA/getAInverse/getM/getR/getMpinv/getFixed/getFree of a fixed
//                              problem (raw doubles) for tests/test_cpp_api.py to compare with the oracle
// Exit status 0 = all checks passed.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mav_trajectory_generation/batch_polynomial_optimization.h"
#include "mav_trajectory_generation/polynomial_optimization_linear.h"

using namespace mav_trajectory_generation;

static int g_fail = 0;
#define EXPECT(cond, ...)                                       \
  do {                                                          \
    if (!(cond)) {                                              \
      ++g_fail;                                                 \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                        \
      std::fprintf(stderr, "\n");                               \
    }                                                           \
  } while (0)

// v << a, b (, c): the Eigen comma initializer, valid with Eigen and with the drop-in's own types
static VectorXd vec(double a, double b) {
  VectorXd v(2);
  v << a, b;
  return v;
}
static VectorXd vec(double a, double b, double c) {
  VectorXd v(3);
  v << a, b, c;
  return v;
}

static double maxabs(const VectorXd& v) {
  double m = 0;
  for (int i = 0; i < (int)v.size(); ++i) m = std::fmax(m, std::fabs(v[i]));
  return m;
}

// checkPath (test_polynomial_optimization.cpp:73-131), tolerance relative to the derivative's scale
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
        const VectorXd actual = s.evaluate(t, it->first);
        const double scale = std::fmax(1.0, maxabs(it->second));
        for (int d = 0; d < s.D(); ++d)
          EXPECT(std::fabs(actual[d] - it->second[d]) <= tol * scale, "fixed constraint seg %zu end %d der %d", i, end,
                 it->first);
      }
    }
    if (i > 0) {
      const Segment& p = segments[i - 1];
      for (int der = 0; der < N / 2; ++der) {
        const VectorXd a = p.evaluate(p.getTime(), der), b = s.evaluate(0.0, der);
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
  const VectorXd c = segments[0][0].getCoefficients();
  for (int j = 0; j < 10; ++j) EXPECT(std::fabs(c[j] - matlab[j]) <= 1e-13, "2_vertices_setup c[%d]", j);
  EXPECT(opt.getNumberFreeConstraints() == 0, "n_free");
  EXPECT(opt.getNumberSegments() == 1, "n_segments");
}

// PathPlanning_A_matrix_inversion (test_polynomial_optimization.cpp:194-204): the static Schur
// inverse of the static mapping matrix, and the exact-table getAInverse, against A
static void test_mapping_matrix_inversion() {
  for (double T = 1.0; T <= 60.0; T += 1.0) {
    PolynomialOptimization<10>::SquareMatrix A, Ai;
    PolynomialOptimization<10>::setupMappingMatrix(T, &A);
    PolynomialOptimization<10>::invertMappingMatrix(A, &Ai);
    MatrixXd P = Ai * A;
    double err = 0.0;
    for (int i = 0; i < 10; ++i)
      for (int j = 0; j < 10; ++j) err = std::fmax(err, std::fabs(P(i, j) - (i == j ? 1.0 : 0.0)));
    EXPECT(err < 1e-10 * std::pow(T, 9), "A^-1 A != I at T=%g (%g)", T, err);
  }
  Vertex::Vector vertices = createRandomVertices(derivative_order::SNAP, 4, vec(-1.0, -1.0), vec(1.0, 1.0), 3);
  const std::vector<double> times = estimateSegmentTimes(vertices, 3.0, 5.0);
  PolynomialOptimization<10> opt(2);
  opt.setupFromVertices(vertices, times);
  MatrixXd A, Ai;
  opt.getA(&A);
  opt.getAInverse(&Ai);
  const MatrixXd P = Ai * A;
  double err = 0.0;
  for (int i = 0; i < P.rows(); ++i)
    for (int j = 0; j < P.cols(); ++j) err = std::fmax(err, std::fabs(P(i, j) - (i == j ? 1.0 : 0.0)));
  EXPECT(err < 1e-9, "getAInverse * getA != I (%g)", err);
}

// createRandomVertices + estimateSegmentTimes, then the single-problem API; checkPath, the
// M / R / Mpinv identities and cost consistency (PathPlanning tests :280-420)
template <int N>
static void test_random_paths(int D, int K, int max_derivative, int r, int seeds, bool device) {
  VectorXd pmin = VectorXd::Constant(D, -10.0), pmax = VectorXd::Constant(D, 10.0);
  for (int seed = 0; seed < seeds; ++seed) {
    Vertex::Vector vertices = createRandomVertices(max_derivative, K, pmin, pmax, 1000 + seed);
    const std::vector<double> times = estimateSegmentTimes(vertices, 3.0, 5.0);
    PolynomialOptimization<N> opt(D);
    opt.setupFromVertices(vertices, times, r);
    opt.solveLinear();
    Segment::Vector segments;
    opt.getSegments(&segments);
    checkPath<N>(vertices, segments, 1e-8);
    const double cost = opt.computeCost();
    EXPECT(std::isfinite(cost) && cost >= 0.0, "cost");
    EXPECT(opt.getNumberAllConstraints() == (size_t)K * N, "all constraints");
    // d^T R d / 2 over all dimensions equals the cost (R = M^T A^-T Q A^-1 M, lin_impl:298-326)
    MatrixXd R, M, Mp;
    opt.getR(&R);
    opt.getM(&M);
    opt.getMpinv(&Mp);
    std::vector<VectorXd> fixed, free;
    opt.getFixedConstraints(&fixed);
    opt.getFreeConstraints(&free);
    const size_t nf = opt.getNumberFixedConstraints(), np = opt.getNumberFreeConstraints();
    EXPECT(R.rows() == (Index)(nf + np) && M.rows() == (Index)(K * N) && Mp.rows() == (Index)(nf + np), "shapes");
    double dRd = 0.0;
    for (int d = 0; d < D; ++d) {
      VectorXd x(nf + np);
      for (size_t i = 0; i < nf; ++i) x[i] = fixed[d][i];
      for (size_t i = 0; i < np; ++i) x[nf + i] = free[d][i];
      const VectorXd Rx = R * x;
      for (size_t i = 0; i < nf + np; ++i) dRd += x[i] * Rx[i];
      // optimality: (R d)_free = 0 (the gradient of the free derivatives vanishes)
      double g = 0.0, sc = 0.0;
      for (size_t i = 0; i < nf + np; ++i) sc = std::fmax(sc, std::fabs(Rx[i]));
      for (size_t i = nf; i < nf + np; ++i) g = std::fmax(g, std::fabs(Rx[i]));
      EXPECT(g <= 1e-6 * sc, "stationarity %g vs %g", g, sc);
    }
    EXPECT(std::fabs(0.5 * dRd - cost) <= 1e-7 * std::fmax(cost, 1e-12), "d^T R d / 2 = %g vs cost %g", 0.5 * dRd,
           cost);
    const MatrixXd MpM = Mp * M;
    double e = 0.0;
    for (int i = 0; i < MpM.rows(); ++i)
      for (int j = 0; j < MpM.cols(); ++j) e = std::fmax(e, std::fabs(MpM(i, j) - (i == j ? 1.0 : 0.0)));
    EXPECT(e == 0.0, "Mpinv * M != I");

    if (device) {  // the batched entry point gives the same coefficients as the single problem on the GPU
      BatchPolynomialOptimization<N> batch(D, K, r);
      std::vector<double> coeffs, bcost;
      batch.solve({vertices}, {times}, &coeffs, &bcost);
      for (int i = 0; i < K; ++i)
        for (int d = 0; d < D; ++d) {
          const VectorXd c = segments[i][d].getCoefficients();
          for (int j = 0; j < N; ++j) EXPECT(c[j] == coeffs[((size_t)i * D + d) * N + j], "batch vs single");
        }
      // (computeCost forms Q with pow() the reference's way, lin_impl:574-589; the kernel's cost uses
      // the exact table: at N = 12 the two differ in the 8th digit)
      EXPECT(std::fabs(bcost[0] - cost) <= 1e-7 * std::fmax(cost, 1e-12), "batch cost %.17g vs %.17g", bcost[0], cost);
      // several devices (here two contexts on device 0: the mtg_solve_linear_batch_multi path, one host
      // thread per context): three copies of the problem, shards of 2 + 1, the same bits
      BatchPolynomialOptimization<N> multi(D, K, r, std::vector<int>{0, 0});
      EXPECT(multi.numDevices() == 2, "two contexts");
      std::vector<double> mcoeffs;
      multi.solve({vertices, vertices, vertices}, {times, times, times}, &mcoeffs);
      const size_t per = (size_t)K * D * N;
      for (size_t b = 0; b < 3; ++b)
        for (size_t q = 0; q < per; ++q) EXPECT(mcoeffs[b * per + q] == coeffs[q], "multi-device batch vs one device");
    }
  }
}

// ConstraintPacking (test_polynomial_optimization.cpp:777-836): counts and (vertex, derivative) order
static void test_constraint_packing() {
  const int K = 5, D = 3;
  Vertex::Vector vertices;
  for (int v = 0; v <= K; ++v) {
    Vertex vx(D);
    if (v == 0 || v == K)
      vx.makeStartOrEnd(vec(1.0 * v, 2.0, 3.0), derivative_order::JERK);
    else
      vx.addConstraint(derivative_order::POSITION, vec(1.0 * v, -1.0 * v, 0.5 * v));
    vertices.push_back(vx);
  }
  PolynomialOptimization<10> opt(D);
  opt.setupFromVertices(vertices, std::vector<double>(K, 1.5), derivative_order::SNAP);
  opt.solveLinear();
  EXPECT(opt.getNumberFixedConstraints() == 2 * 4 + (K - 1), "n_fixed %zu", opt.getNumberFixedConstraints());
  EXPECT(opt.getNumberFreeConstraints() == 2 * 1 + (K - 1) * 4, "n_free %zu", opt.getNumberFreeConstraints());
  std::vector<VectorXd> fc, fx;
  opt.getFreeConstraints(&fc);
  opt.getFixedConstraints(&fx);
  EXPECT(fc.size() == (size_t)D && (size_t)fc[0].size() == opt.getNumberFreeConstraints(), "free shape");
  // fixed values in (vertex, derivative) order: vertex 0's position, 3 zero derivatives, then the
  // interior positions, then the last vertex
  EXPECT(fx[0][0] == 0.0 && fx[1][0] == 2.0 && fx[0][4] == 1.0 && fx[2][5] == 1.0, "fixed order");
  // the first free value is vertex 0's snap
  Segment::Vector segments;
  opt.getSegments(&segments);
  for (int d = 0; d < D; ++d)
    EXPECT(std::fabs(segments[0].evaluate(0.0, derivative_order::SNAP)[d] - fc[d][0]) <=
               1e-9 * std::fmax(1.0, std::fabs(fc[d][0])),
           "free snap at vertex 0, dim %d", d);
}

// evaluateRange: count, times and values against per-sample Trajectory::evaluate; the maximum speed
// (computeMaximumOfMagnitude, host roots) against sampling
static void test_evaluate_range(bool device) {
  Vertex::Vector vertices;
  for (int v = 0; v <= 3; ++v) {
    Vertex vx(2);
    if (v == 0 || v == 3)
      vx.makeStartOrEnd(vec(1.0 * v, -2.0 * v), derivative_order::SNAP);
    else
      vx.addConstraint(derivative_order::POSITION, vec(1.0 * v + 0.3, 0.7 * v));
    vertices.push_back(vx);
  }
  PolynomialOptimization<10> opt(2);
  opt.setupFromVertices(vertices, {1.0, 2.0, 1.5});
  opt.solveLinear();
  Trajectory traj;
  opt.getTrajectory(&traj);
  std::vector<VectorXd> samples;
  std::vector<double> st;
  traj.evaluateRange(0.0, traj.getMaxTime(), 0.01, derivative_order::POSITION, &samples, &st);
  EXPECT(samples.size() == st.size() && samples.size() >= 449 && samples.size() <= 451, "samples %zu", samples.size());
  for (size_t s = 0; s < samples.size(); s += 37) {
    const VectorXd e = traj.evaluate(st[s], derivative_order::POSITION);
    for (int d = 0; d < 2; ++d)
      EXPECT(std::fabs(e[d] - samples[s][d]) <= 1e-12 * std::fmax(1.0, std::fabs(e[d])), "sample %zu", s);
  }
  std::vector<VectorXd> vel;
  traj.evaluateRange(0.0, traj.getMaxTime(), 0.001, derivative_order::VELOCITY, &vel);
  double smax = 0.0;
  for (const VectorXd& v : vel) smax = std::fmax(smax, v.norm());
  std::vector<Extremum> cands;
  const Extremum vmax_h = opt.computeMaximumOfMagnitude<derivative_order::VELOCITY>(&cands);
  EXPECT(vmax_h.value >= smax * (1 - 1e-12) && vmax_h.value <= smax * (1 + 1e-4), "max speed %g vs sampled %g",
         vmax_h.value, smax);
  EXPECT(cands.size() >= 4, "candidates %zu", cands.size());
  if (device) {
    // the same samples through the GPU kernels, and computeMinMaxMagnitude (trajectory.cpp:185-218)
    std::vector<VectorXd> samples_d;
    std::vector<double> st_d;
    traj.evaluateRangeDevice(0.0, traj.getMaxTime(), 0.01, derivative_order::POSITION, &samples_d, &st_d);
    EXPECT(samples_d.size() == samples.size(), "device sample count");
    bool same = samples_d.size() == samples.size();
    for (size_t s = 0; same && s < samples.size(); ++s) same = samples_d[s] == samples[s] && st_d[s] == st[s];
    EXPECT(same, "device evaluateRange bits");
    Extremum vmin, vmax;
    EXPECT(traj.computeMinMaxMagnitude(derivative_order::VELOCITY, {0, 1}, &vmin, &vmax), "min/max magnitude");
    EXPECT(vmax.value >= smax * (1 - 1e-12) && vmax.value <= smax * (1 + 1e-4), "max speed %g vs sampled %g",
           vmax.value, smax);
    EXPECT(std::fabs(vmax.value - vmax_h.value) <= 1e-9 * vmax.value, "GPU vs host maximum %g %g", vmax.value,
           vmax_h.value);
    EXPECT(vmin.value <= 1e-9 && vmax.segment_idx >= 0 && vmax.segment_idx < 3, "min speed %g (rest at the ends)",
           vmin.value);
  }
}

// error behaviour: CHECKs of setupFromVertices (lin_impl:50-55, :66-67, :287) as Error here
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
  // constraints above N/2-1 are dropped with a warning (lin_impl:74-95)
  PolynomialOptimization<8> opt8(1);
  opt8.setupFromVertices(vertices, {1.0}, 3);
  EXPECT(opt8.getNumberFixedConstraints() == 8, "orders > 3 dropped for N=8");
}

// setFreeConstraints round trip and computeInitialSolutionWithoutPositionConstraints (nl_impl:116-187)
static void test_free_constraints_and_reparametrisation() {
  const int K = 6, D = 3, N = 10;
  Vertex::Vector vertices;
  for (int v = 0; v <= K; ++v) {
    Vertex vx(D);
    if (v == 0 || v == K)
      vx.makeStartOrEnd(vec(1.0 * v, 2.0 - v, 0.5), derivative_order::SNAP);
    else
      vx.addConstraint(derivative_order::POSITION, vec(1.0 * v + 0.2 * (v % 2), -0.7 * v, 0.3 * v * v));
    vertices.push_back(vx);
  }
  std::vector<double> times{1.1, 0.8, 1.7, 2.2, 0.9, 1.3};
  PolynomialOptimization<N> opt(D);
  opt.setupFromVertices(vertices, times, derivative_order::SNAP);
  opt.solveLinear();
  Segment::Vector s0;
  opt.getSegments(&s0);
  const double cost0 = opt.computeCost();
  std::vector<VectorXd> fc, fx;
  opt.getFreeConstraints(&fc);
  opt.getFixedConstraints(&fx);
  EXPECT(fx.size() == (size_t)D && (size_t)fx[0].size() == opt.getNumberFixedConstraints(), "fixed shape");
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

// The matrices of one fixed problem, for tests/test_cpp_api.py to compare with the oracle's.
static int dump(const char* path) {
  Vertex::Vector vertices =
      createRandomVertices(derivative_order::SNAP, 5, vec(-10.0, -20.0, -10.0), vec(10.0, 20.0, 10.0), 12345);
  vertices[2].addConstraint(derivative_order::VELOCITY, vec(0.5, -0.25, 1.0));  // a mixed mask
  const std::vector<double> times = estimateSegmentTimes(vertices, 3.0, 5.0);
  PolynomialOptimization<10> opt(3);
  opt.setupFromVertices(vertices, times, derivative_order::SNAP);
  opt.solveLinear();
  MatrixXd A, Ai, M, R, Mp;
  opt.getA(&A);
  opt.getAInverse(&Ai);
  opt.getM(&M);
  opt.getR(&R);
  opt.getMpinv(&Mp);
  std::vector<VectorXd> fixed, free;
  opt.getFixedConstraints(&fixed);
  opt.getFreeConstraints(&free);
  FILE* f = std::fopen(path, "wb");
  if (!f) return 2;
  auto put = [&](const MatrixXd& m) {  // rows, cols, row-major values
    const double hdr[2] = {(double)m.rows(), (double)m.cols()};
    std::fwrite(hdr, sizeof(double), 2, f);
    for (Index i = 0; i < m.rows(); ++i)
      for (Index j = 0; j < m.cols(); ++j) {
        const double x = m(i, j);
        std::fwrite(&x, sizeof(double), 1, f);
      }
  };
  put(A), put(Ai), put(M), put(R), put(Mp);
  MatrixXd fx(3, fixed[0].size()), fr(3, free[0].size()), tm(1, (Index)times.size()), c(1, 1);
  for (int d = 0; d < 3; ++d) {
    for (Index i = 0; i < fixed[d].size(); ++i) fx(d, i) = fixed[d][i];
    for (Index i = 0; i < free[d].size(); ++i) fr(d, i) = free[d][i];
  }
  for (size_t i = 0; i < times.size(); ++i) tm(0, (Index)i) = times[i];
  c(0, 0) = opt.computeCost();
  put(fx), put(fr), put(tm), put(c);
  std::fclose(f);
  return 0;
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "host";
  if (mode == "dump") return argc > 2 ? dump(argv[2]) : 2;
  const bool device = mode == "device";
  setExecutionPolicy(device ? ExecutionPolicy::kDevice : ExecutionPolicy::kHost);
  test_free_constraints_and_reparametrisation();
  test_two_vertices_setup();
  test_mapping_matrix_inversion();
  test_random_paths<10>(3, 10, 4, 4, 20, device);
  test_random_paths<8>(2, 6, 3, 2, 10, device);
  test_random_paths<12>(3, 20, 4, 3, 5, device);
  test_random_paths<12>(1, 15, 4, 3, 3, device);
  test_constraint_packing();
  test_evaluate_range(device);
  test_errors();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("test_cpp_api (%s): all checks passed\n", mode.c_str());
  return 0;
}
