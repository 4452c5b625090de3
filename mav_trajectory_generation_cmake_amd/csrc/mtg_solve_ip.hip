// mtg_solve_ip.hip -- dispatch of the interior-waypoint lane kernel (mtg_solve_ip.inc; one
// translation unit per N in mtg_solve_ip_n*.hip).
#include "mtg_solve_ip.inc"  // (templates only: no kernel is instantiated in this unit)

namespace mtg {

hipError_t launch_solve_ip_n6(const SolveArgs&, hipStream_t);
hipError_t launch_solve_ip_n8(const SolveArgs&, hipStream_t);
hipError_t launch_solve_ip_n10(const SolveArgs&, hipStream_t);
hipError_t launch_solve_ip_n12(const SolveArgs&, hipStream_t);

// Shapes the kernel serves (IpShape<N, K, D>::OK at run time): N in {6, 8, 10, 12}, D <= 4,
// K in {4, 8, 10, 12} (a register bucket of the column kernel, which runs the waves of other
// patterns), r >= 1 (translation-relative positions), and the lane's state within budget.
bool ip_geometry(int N, int D, int K, int r) {
  if (N < 6 || N > 12 || (N % 2) || D < 1 || D > 4 || r < 1 || r > N / 2 - 1) return false;
  if (K != 4 && K != 8 && K != 10 && K != 12) return false;
  const int H = N / 2, F = H - 1, KC = K / 2, KS = KC - 1, NL = F * (F - 1) / 2;
  if (KS * (NL + F + D * F) + KC > 110 || H * K > 50) return false;
  int lg;
  size_t lds;
  if (!reg_geometry(N, D, K, &lg, &lds)) return false;
  return sizeof(double) * (size_t)ip_lds_doubles(N, D, K) <= kMaxLdsPerBlock;
}

hipError_t launch_solve_ip(int N, const SolveArgs& a, hipStream_t stream) {
  if (!ip_geometry(N, a.D, a.K, a.r)) return hipErrorInvalidValue;
  switch (N) {
    case 6: return launch_solve_ip_n6(a, stream);
    case 8: return launch_solve_ip_n8(a, stream);
    case 10: return launch_solve_ip_n10(a, stream);
    case 12: return launch_solve_ip_n12(a, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
