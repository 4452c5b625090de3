// mtg_solve_dl.hip -- dispatch of the dimension-lane kernel (mtg_solve_dl.inc; one translation unit
// per (N, D) in mtg_solve_dl_n*_d*.hip).
#include "mtg_solve_dl.inc"  // (templates only: no kernel is instantiated in this unit)

namespace mtg {

#define MTG_DL_DECL(NN, DD) hipError_t launch_solve_dl_n##NN##_d##DD(const SolveArgs&, hipStream_t);
MTG_DL_DECL(10, 1) MTG_DL_DECL(10, 2) MTG_DL_DECL(10, 3) MTG_DL_DECL(10, 4)
MTG_DL_DECL(12, 1) MTG_DL_DECL(12, 2) MTG_DL_DECL(12, 3) MTG_DL_DECL(12, 4)
#undef MTG_DL_DECL

// Shapes the kernel serves: N = 10 with K = 10 (configs 2, 3) and N = 12 with K = 20 (config 4),
// D <= 4, r >= 1 (translation-relative positions); its LDS (and the general kernel's block function's,
// for the trajectories of other patterns) within a CU's 160 KB.
bool dl_geometry(int N, int D, int K, int r) {
  if (D < 1 || D > 4 || r < 1 || r > N / 2 - 1 || K != dl_kmax(N) || K == 0) return false;
  size_t lds = 0;
#define MTG_DL_LDS(NN, DD) \
  if (N == NN && D == DD) lds = dl_lds_bytes<NN, DD>();
  MTG_DL_LDS(10, 1) MTG_DL_LDS(10, 2) MTG_DL_LDS(10, 3) MTG_DL_LDS(10, 4)
  MTG_DL_LDS(12, 1) MTG_DL_LDS(12, 2) MTG_DL_LDS(12, 3) MTG_DL_LDS(12, 4)
#undef MTG_DL_LDS
  return lds > 0 && lds <= kMaxLdsHard;
}

hipError_t launch_solve_dl(int N, const SolveArgs& a, hipStream_t stream) {
  if (!dl_geometry(N, a.D, a.K, a.r)) return hipErrorInvalidValue;
#define MTG_DL_CASE(NN, DD) \
  if (N == NN && a.D == DD) return launch_solve_dl_n##NN##_d##DD(a, stream);
  MTG_DL_CASE(10, 1) MTG_DL_CASE(10, 2) MTG_DL_CASE(10, 3) MTG_DL_CASE(10, 4)
  MTG_DL_CASE(12, 1) MTG_DL_CASE(12, 2) MTG_DL_CASE(12, 3) MTG_DL_CASE(12, 4)
#undef MTG_DL_CASE
  return hipErrorInvalidValue;
}

}  // namespace mtg
