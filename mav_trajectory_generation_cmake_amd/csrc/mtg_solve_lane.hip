// mtg_solve_lane.hip -- dispatch of the lane-per-chain solve kernel (mtg_solve_lane.inc; one
// translation unit per (N, D) in mtg_solve_lane_n*_d*.hip).
#include "mtg_solve_lane.inc"  // (templates only: no kernel is instantiated in this unit)

namespace mtg {

#define MTG_LANE_DECL(NN, DD) hipError_t launch_solve_lane_n##NN##_d##DD(const SolveArgs&, size_t, hipStream_t);
MTG_LANE_DECL(6, 1) MTG_LANE_DECL(6, 2) MTG_LANE_DECL(6, 3) MTG_LANE_DECL(6, 4)
MTG_LANE_DECL(8, 1) MTG_LANE_DECL(8, 2) MTG_LANE_DECL(8, 3) MTG_LANE_DECL(8, 4)
MTG_LANE_DECL(10, 1) MTG_LANE_DECL(10, 2) MTG_LANE_DECL(10, 3) MTG_LANE_DECL(10, 4)
#undef MTG_LANE_DECL

// N in {6, 8, 10}, D <= 4, K <= 12 with h^2 KMAX/2 <= kLaneGMax doubles of G per lane, and the
// LDS of 32 trajectories within 64 KB.
bool lane_geometry(int N, int D, int K, size_t* lds_bytes) {
  if (N != 6 && N != 8 && N != 10) return false;
  if (D < 1 || D > 4) return false;
  const int km = reg_kmax(K), H = N / 2;
  if (km < 0 || km > kRegKMax || H * H * (km / 2) > kLaneGMax) return false;
  const size_t bytes = (size_t)lane_lds_doubles(N, D, K) * sizeof(double);
  if (bytes > kMaxLdsPerBlock) return false;
  *lds_bytes = bytes;
  return true;
}

hipError_t launch_solve_lane(int N, const SolveArgs& a, hipStream_t stream) {
  size_t lds;
  if (!lane_geometry(N, a.D, a.K, &lds)) return hipErrorInvalidValue;
#define MTG_LANE_CASE(NN, DD) \
  if (N == NN && a.D == DD) return launch_solve_lane_n##NN##_d##DD(a, lds, stream);
  MTG_LANE_CASE(6, 1) MTG_LANE_CASE(6, 2) MTG_LANE_CASE(6, 3) MTG_LANE_CASE(6, 4)
  MTG_LANE_CASE(8, 1) MTG_LANE_CASE(8, 2) MTG_LANE_CASE(8, 3) MTG_LANE_CASE(8, 4)
  MTG_LANE_CASE(10, 1) MTG_LANE_CASE(10, 2) MTG_LANE_CASE(10, 3) MTG_LANE_CASE(10, 4)
#undef MTG_LANE_CASE
  return hipErrorInvalidValue;
}

}  // namespace mtg
