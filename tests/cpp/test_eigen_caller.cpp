// A caller written the way the reference's own code calls PolynomialOptimization<N>: Eigen types
// in and out (Eigen::VectorXd constraints into makeStartOrEnd / addConstraint, Eigen::MatrixXd out
// of getR, std::vector<Eigen::VectorXd> out of getFreeConstraints), as in the reference's benchmark
// (src/polynomial_timing_evaluation.cpp:34-91, :93-128) and its tests
// (test/test_polynomial_optimization.cpp).  It is compiled against the drop-in headers in their
// Eigen mode (tests/test_eigen_api.py: -I tests/eigen_shim, a test-only Eigen stand-in, since the
// image has no Eigen) and checks itself against the library's C ABI on the same problems.
// Exit status 0 and "all checks passed" on success.
#include <cmath>
#include <cstdio>
#include <random>
#include <type_traits>
#include <vector>

#include <eigen3/Eigen/Core>
#include <mav_trajectory_generation/polynomial_optimization_linear.h>

#ifndef MTG_USE_EIGEN
#error "the drop-in headers did not select their Eigen mode"
#endif

namespace mtg = mav_trajectory_generation;

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

// The benchmark's vertex path (the reference's createRandomVerticesPath, restated with Eigen as its
// callers write it): directions U(-1, 1)^D rejected below 0.2, normalised and scaled by
// U(0, 2 average_distance); the offset is kept as the next "last position", and the end vertex fixes
// the last offset up to max_derivative.
static mtg::Vertex::Vector pathWithEigen(int dimension, int n_segments, double average_distance, int max_derivative,
                                         unsigned seed) {
  std::mt19937 generator(seed);
  std::vector<std::uniform_real_distribution<double>> direction(dimension,
                                                                std::uniform_real_distribution<double>(-1, 1));
  std::uniform_real_distribution<double> distance(0, 2 * average_distance);
  mtg::Vertex::Vector vertices;
  Eigen::VectorXd last(dimension);
  for (int d = 0; d < dimension; ++d) last[d] = direction[d](generator);
  vertices.push_back(mtg::Vertex(dimension));
  vertices.front().makeStartOrEnd(last, max_derivative);
  for (int i = 1; i <= n_segments; ++i) {
    Eigen::VectorXd step(dimension);
    do {
      for (int d = 0; d < dimension; ++d) step[d] = direction[d](generator);
    } while (!(step.norm() > 0.2));
    step = step.normalized() * distance(generator);
    mtg::Vertex v(dimension);
    v.addConstraint(mtg::derivative_order::POSITION, step + last);
    vertices.push_back(v);
    last = step;
  }
  vertices.back().makeStartOrEnd(last, max_derivative);
  return vertices;
}

static void check_path_against_abi(int K, unsigned seed) {
  const int N = 10, D = 3, h = N / 2, V = K + 1;
  const mtg::Vertex::Vector vertices = pathWithEigen(D, K, 5.0, mtg::derivative_order::SNAP, seed);
  const std::vector<double> times = mtg::estimateSegmentTimes(vertices, 2.0, 2.0, 6.5);

  // the library's own generator of the benchmark's problems must give the same bits
  std::vector<double> values((size_t)V * h * D), t((size_t)K);
  std::vector<uint8_t> mask((size_t)V);
  EXPECT(mtg_host_random_vertices_path_batch(N, D, K, 5.0, mtg::derivative_order::SNAP, seed, 1, 2.0, 2.0, 6.5,
                                             values.data(), mask.data(), t.data(), 1) == MTG_OK,
         "generator");
  for (int v = 0; v < V; ++v) {
    Eigen::VectorXd p;
    EXPECT(vertices[v].getConstraint(mtg::derivative_order::POSITION, &p), "position of vertex %d", v);
    for (int d = 0; d < D; ++d) EXPECT(p[d] == values[(size_t)v * h * D + d], "vertex %d dim %d bits", v, d);
  }
  for (int i = 0; i < K; ++i) EXPECT(times[i] == t[i], "segment time %d bits", i);

  // the reference's sequence: setupFromVertices, solveLinear, then the accessors with Eigen types
  mtg::PolynomialOptimization<N> opt(D);
  opt.setupFromVertices(vertices, times, mtg::derivative_order::SNAP);
  opt.solveLinear();
  std::vector<Eigen::VectorXd> free_constraints, fixed_constraints;
  opt.getFreeConstraints(&free_constraints);
  opt.getFixedConstraints(&fixed_constraints);
  Eigen::MatrixXd R;
  opt.getR(&R);
  mtg::Segment::Vector segments;
  opt.getSegments(&segments);
  const double cost = opt.computeCost();

  // the same problem through the C ABI's host solver: identical bits
  std::vector<double> coeffs((size_t)K * D * N), free_out((size_t)D * V * h), cost_abi(1);
  int32_t n_free = 0, status = -1;
  EXPECT(mtg_host_solve_linear_batch(N, D, K, mtg::derivative_order::SNAP, 1, values.data(), mask.data(), t.data(),
                                     coeffs.data(), free_out.data(), &n_free, cost_abi.data(), &status, 1) == MTG_OK,
         "host solve");
  EXPECT(status == 0 && (size_t)n_free == opt.getNumberFreeConstraints(), "status %d n_free %d", status, n_free);
  for (int i = 0; i < K; ++i)
    for (int d = 0; d < D; ++d) {
      const Eigen::VectorXd c = segments[i][d].getCoefficients();
      for (int j = 0; j < N; ++j) EXPECT(c[j] == coeffs[((size_t)i * D + d) * N + j], "coefficient %d %d %d", i, d, j);
    }
  for (int d = 0; d < D; ++d)
    for (int k = 0; k < n_free; ++k) EXPECT(free_constraints[d][k] == free_out[(size_t)d * V * h + k], "free %d %d", d, k);

  // R is M^T A^-T Q A^-1 M: d^T R d / 2 over the dimensions is the cost, and R's free rows vanish at
  // the optimum (the reference's normal equations R_pp d_p = -R_pf d_f, lin_impl:341-365)
  const Eigen::Index nf = (Eigen::Index)opt.getNumberFixedConstraints(), np = (Eigen::Index)opt.getNumberFreeConstraints();
  EXPECT(R.rows() == nf + np && R.cols() == nf + np, "R shape");
  double dRd = 0.0;
  for (int d = 0; d < D; ++d) {
    Eigen::VectorXd x(nf + np);
    for (Eigen::Index i = 0; i < nf; ++i) x[i] = fixed_constraints[d][i];
    for (Eigen::Index i = 0; i < np; ++i) x[nf + i] = free_constraints[d][i];
    const Eigen::VectorXd Rx = R * x;
    dRd += x.dot(Rx);
    const Eigen::VectorXd grad = Rx.tail(np);
    EXPECT(grad.cwiseAbs().maxCoeff() <= 1e-6 * Rx.cwiseAbs().maxCoeff(), "stationarity, dim %d", d);
  }
  EXPECT(std::fabs(0.5 * dRd - cost) <= 1e-7 * cost, "d^T R d / 2 = %.17g vs cost %.17g", 0.5 * dRd, cost);
  EXPECT(std::fabs(cost - cost_abi[0]) <= 1e-7 * cost, "computeCost %.17g vs ABI %.17g", cost, cost_abi[0]);

  // Trajectory / evaluate with Eigen results: continuity at the interior vertices
  mtg::Trajectory trajectory;
  opt.getTrajectory(&trajectory);
  double t_acc = 0.0;
  for (int i = 0; i + 1 < K; ++i) {
    t_acc += times[i];
    for (int der = 0; der < h; ++der) {
      const Eigen::VectorXd a = segments[i].evaluate(times[i], der), b = segments[i + 1].evaluate(0.0, der);
      EXPECT((a - b).norm() <= 1e-6 * std::fmax(1.0, a.norm()), "continuity at vertex %d, derivative %d", i + 1, der);
    }
    const Eigen::VectorXd p = trajectory.evaluate(t_acc - 0.5 * times[i], mtg::derivative_order::POSITION);
    EXPECT(p.size() == D && p.allFinite(), "Trajectory::evaluate");
  }
}

// The reference's 2_vertices_setup known answer (test_polynomial_optimization.cpp:700-744) with
// the Eigen comma initializer
static void two_vertices_setup() {
  mtg::Vertex start(1), end(1);
  Eigen::VectorXd p0(1), p1(1);
  p0 << 0.0;
  p1 << 5.0;
  start.makeStartOrEnd(p0, mtg::derivative_order::SNAP);
  end.makeStartOrEnd(p1, mtg::derivative_order::SNAP);
  mtg::Vertex::Vector vertices{start, end};
  mtg::PolynomialOptimization<10> opt(1);
  opt.setupFromVertices(vertices, {5.0}, mtg::derivative_order::SNAP);
  opt.solveLinear();
  mtg::Segment::Vector segments;
  opt.getSegments(&segments);
  Eigen::VectorXd matlab(10);
  matlab << -0.000000000000004, 0.000000000000004, -0.000000000000006, 0.000000000000003, -0.000000000000001,
      0.201600000000015, -0.134400000000012, 0.034560000000004, -0.004032000000000, 0.000179200000000;
  const Eigen::VectorXd c = segments[0][0].getCoefficients();
  EXPECT((c - matlab).cwiseAbs().maxCoeff() <= 1e-13, "2_vertices_setup coefficients");
  // the static mapping-matrix helpers on Eigen fixed-size matrices (PathPlanning_A_matrix_inversion)
  mtg::PolynomialOptimization<10>::SquareMatrix A, A_inv;
  mtg::PolynomialOptimization<10>::setupMappingMatrix(5.0, &A);
  mtg::PolynomialOptimization<10>::invertMappingMatrix(A, &A_inv);
  const Eigen::MatrixXd I = A_inv * A;
  EXPECT((I - Eigen::MatrixXd::Identity(10, 10)).cwiseAbs().maxCoeff() < 1e-10 * std::pow(5.0, 9), "A^-1 A");
  // the container type spelled out as the reference declares it (polynomial_optimization_linear.h:53-54)
  typedef mtg::PolynomialOptimization<10>::SquareMatrix SM;
  static_assert(std::is_same<mtg::PolynomialOptimization<10>::SquareMatrixVector,
                             std::vector<SM, Eigen::aligned_allocator<SM>>>::value,
                "SquareMatrixVector is std::vector<SquareMatrix, Eigen::aligned_allocator<SquareMatrix>>");
  std::vector<SM, Eigen::aligned_allocator<SM>> inverses(3);
  for (int i = 0; i < 3; ++i) {
    mtg::PolynomialOptimization<10>::setupMappingMatrix(1.0 + i, &A);
    mtg::PolynomialOptimization<10>::invertMappingMatrix(A, &inverses[i]);
  }
  mtg::PolynomialOptimization<10>::SquareMatrixVector same = inverses;
  EXPECT(same.size() == 3 && (same[2] - inverses[2]).cwiseAbs().maxCoeff() == 0.0, "SquareMatrixVector copy");
}

int main() {
  mtg::setExecutionPolicy(mtg::ExecutionPolicy::kHost);
  two_vertices_setup();
  for (unsigned seed = 0; seed < 8; ++seed) check_path_against_abi(10, seed);
  check_path_against_abi(2, 99);
  check_path_against_abi(25, 7);
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("test_eigen_caller: all checks passed\n");
  return 0;
}
