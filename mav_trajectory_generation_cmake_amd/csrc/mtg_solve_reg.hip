// mtg_solve_reg.hip -- dispatch of the register-resident solve kernel (mtg_solve_reg.inc; one
// translation unit per N in mtg_solve_reg_n*.hip).
#include "mtg_solve_reg.inc"  // (templates only: no kernel is instantiated in this unit)

namespace mtg {

hipError_t launch_solve_reg_n2(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n4(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n6(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n8(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n10(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n12(const SolveArgs&, int, size_t, hipStream_t);


bool reg_geometry(int N, int D, int K, int* lanes_per_traj, size_t* lds_bytes) {
  const int H = N / 2;
  // G_v columns take H * KMAX doubles per lane: beyond ~50 the 2-waves-per-SIMD kernel spills
  // (N=12, K > 8); the wide bucket (N = 12, K <= 20) keeps G in LDS instead (Forward::GLDS)
  const int km = reg_kmax(K);
  if (km < 0 || (H * km > 50 && !(N == 12 && km == kRegKMaxWide))) return false;
  int lc = 8;  // lanes per chain: h column lanes + D dimension lanes
  while (lc < H + D) lc *= 2;
  const int lg = kTwist ? 2 * lc : lc;  // twisted: two chains per trajectory
  if (lg > 64) return false;
  const size_t bytes = (size_t)reg_lds_doubles(N, D, K, lg, kTwist) * sizeof(double);
  if (bytes > kMaxLdsPerBlock) return false;
  *lanes_per_traj = lg;
  *lds_bytes = bytes;
  return true;
}

hipError_t launch_solve_reg(int N, const SolveArgs& a, hipStream_t stream) {
  int lg;
  size_t lds;
  if (!reg_geometry(N, a.D, a.K, &lg, &lds)) return hipErrorInvalidValue;
  switch (N) {
    case 2: return launch_solve_reg_n2(a, lg, lds, stream);
    case 4: return launch_solve_reg_n4(a, lg, lds, stream);
    case 6: return launch_solve_reg_n6(a, lg, lds, stream);
    case 8: return launch_solve_reg_n8(a, lg, lds, stream);
    case 10: return launch_solve_reg_n10(a, lg, lds, stream);
    case 12: return launch_solve_reg_n12(a, lg, lds, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
