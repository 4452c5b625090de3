// mtg_solve_dl.hip -- dispatch of the dimension-lane kernel (mtg_solve_dl.inc; one translation unit
// per (N, D) in mtg_solve_dl_n*_d*.hip).
#include "mtg_solve_dl.inc"  // (templates only: no kernel is instantiated in this unit)

namespace mtg {

#define MTG_DL_DECL(NN, DD) hipError_t launch_solve_dl_n##NN##_d##DD(const SolveArgs&, hipStream_t);
MTG_DL_DECL(10, 1) MTG_DL_DECL(10, 2) MTG_DL_DECL(10, 3) MTG_DL_DECL(10, 4)
#undef MTG_DL_DECL

// Shapes the kernel serves: N = 10, K = 10, D <= 4, r >= 1 (translation-relative positions), within
// 64 KB of LDS for its own path and for the general kernel's block function (the waves of other
// patterns).
bool dl_geometry(int N, int D, int K, int r) {
  if (N != 10 || K != 10 || D < 1 || D > 4 || r < 1 || r > N / 2 - 1) return false;
  const size_t fb = sizeof(double) * (size_t)kDlFallbackTraj * slot_doubles(N / 2, D, K, 1 << kDlFallbackLgLog2);
  return sizeof(double) * (size_t)dl_lds_doubles(N, D, K) <= kMaxLdsPerBlock && fb <= kMaxLdsPerBlock;
}

hipError_t launch_solve_dl(int N, const SolveArgs& a, hipStream_t stream) {
  if (!dl_geometry(N, a.D, a.K, a.r)) return hipErrorInvalidValue;
#define MTG_DL_CASE(NN, DD) \
  if (N == NN && a.D == DD) return launch_solve_dl_n##NN##_d##DD(a, stream);
  MTG_DL_CASE(10, 1) MTG_DL_CASE(10, 2) MTG_DL_CASE(10, 3) MTG_DL_CASE(10, 4)
#undef MTG_DL_CASE
  return hipErrorInvalidValue;
}

}  // namespace mtg
