// mtg_solve_dlx.hip -- dispatch of the long-chain dimension-lane kernel (mtg_solve_dlx.inc; one
// translation unit per (N, D) in mtg_solve_dlx_n*_d*.hip).
#include "mtg_solve_dlx.inc"  // (templates only: no kernel is instantiated in this unit)

namespace mtg {

#define MTG_DLX_DECL(NN, DD)                                                   \
  hipError_t launch_solve_dlx_n##NN##_d##DD(const SolveArgs&, hipStream_t); \
  int64_t dlx_resident_slots_n##NN##_d##DD();                               \
  int dlx_tpw_n##NN##_d##DD(int64_t B);
MTG_DLX_DECL(6, 1) MTG_DLX_DECL(6, 2) MTG_DLX_DECL(6, 3) MTG_DLX_DECL(6, 4)
  MTG_DLX_DECL(8, 1) MTG_DLX_DECL(8, 2) MTG_DLX_DECL(8, 3) MTG_DLX_DECL(8, 4)
  MTG_DLX_DECL(10, 1) MTG_DLX_DECL(10, 2) MTG_DLX_DECL(10, 3) MTG_DLX_DECL(10, 4)
MTG_DLX_DECL(12, 1) MTG_DLX_DECL(12, 2) MTG_DLX_DECL(12, 3) MTG_DLX_DECL(12, 4)
#undef MTG_DLX_DECL

// Shapes the kernel serves: N = 6 .. 12, D <= 4, r >= 1 (translation-relative positions), K >= 2, where
// neither the fixed-length DL kernel (N = 10 / 12: K = 10 / 20) nor the register column kernel (N = 6 /
// 8: K <= 12; N = 10: K <= 10; N = 12: K <= 20) applies, and only where the general kernel's geometry
// exists (it solves the complement).
bool dlx_geometry(int N, int D, int K, int r) {
  if (N < 6 || N > 12 || (N % 2) || D < 1 || D > 4 || r < 1 || r > N / 2 - 1 || K < 2) return false;
  int lg, tpb;
  size_t lds;
  if (dl_geometry(N, D, K, r) || reg_geometry(N, D, K, &lg, &lds)) return false;
  return solve_geometry(N, D, K, &lg, &lds, &tpb);
}

static int64_t dlx_rec_doubles(int N, int D) {
  switch (N * 8 + D) {
#define MTG_DLX_REC(NN, DD) \
  case NN * 8 + DD: return DlxShape<NN, DD>::REC;
    MTG_DLX_REC(6, 1) MTG_DLX_REC(6, 2) MTG_DLX_REC(6, 3) MTG_DLX_REC(6, 4)
  MTG_DLX_REC(8, 1) MTG_DLX_REC(8, 2) MTG_DLX_REC(8, 3) MTG_DLX_REC(8, 4)
  MTG_DLX_REC(10, 1) MTG_DLX_REC(10, 2) MTG_DLX_REC(10, 3) MTG_DLX_REC(10, 4)
    MTG_DLX_REC(12, 1) MTG_DLX_REC(12, 2) MTG_DLX_REC(12, 3) MTG_DLX_REC(12, 4)
#undef MTG_DLX_REC
    default: return 0;
  }
}

// Workspace of one launch over B trajectories (pairs): one wave slot per resident wave, at most one per
// wave of work, each slot KB = K - K/2 records; then one 32-bit word per wave of work (which of its
// trajectories the rest kernel solves).
size_t dlx_workspace_bytes(int N, int D, int K, int64_t B) {
  if (B <= 0 || !dlx_geometry(N, D, K, 1)) return 0;
  int64_t resident = 0;
  int tpw = 0;
#define MTG_DLX_RES(NN, DD) \
  if (N == NN && D == DD) resident = dlx_resident_slots_n##NN##_d##DD(), tpw = dlx_tpw_n##NN##_d##DD(B);
  MTG_DLX_RES(6, 1) MTG_DLX_RES(6, 2) MTG_DLX_RES(6, 3) MTG_DLX_RES(6, 4)
  MTG_DLX_RES(8, 1) MTG_DLX_RES(8, 2) MTG_DLX_RES(8, 3) MTG_DLX_RES(8, 4)
  MTG_DLX_RES(10, 1) MTG_DLX_RES(10, 2) MTG_DLX_RES(10, 3) MTG_DLX_RES(10, 4)
  MTG_DLX_RES(12, 1) MTG_DLX_RES(12, 2) MTG_DLX_RES(12, 3) MTG_DLX_RES(12, 4)
#undef MTG_DLX_RES
  if (resident <= 0 || tpw <= 0) return 0;
  const int64_t tasks = (B + tpw - 1) / tpw;
  const int64_t slots = tasks < resident ? tasks : resident;
  const size_t rest = (size_t)((tasks * 4 + 255) / 256 * 256);  // the per-wave rest bits, at the end
  return (size_t)slots * (size_t)(K - K / 2) * (size_t)dlx_rec_doubles(N, D) * sizeof(double) + rest;
}

hipError_t launch_solve_dlx(int N, const SolveArgs& a, hipStream_t stream) {
  if (!dlx_geometry(N, a.D, a.K, a.r)) return hipErrorInvalidValue;
#define MTG_DLX_CASE(NN, DD) \
  if (N == NN && a.D == DD) return launch_solve_dlx_n##NN##_d##DD(a, stream);
  MTG_DLX_CASE(6, 1) MTG_DLX_CASE(6, 2) MTG_DLX_CASE(6, 3) MTG_DLX_CASE(6, 4)
  MTG_DLX_CASE(8, 1) MTG_DLX_CASE(8, 2) MTG_DLX_CASE(8, 3) MTG_DLX_CASE(8, 4)
  MTG_DLX_CASE(10, 1) MTG_DLX_CASE(10, 2) MTG_DLX_CASE(10, 3) MTG_DLX_CASE(10, 4)
  MTG_DLX_CASE(12, 1) MTG_DLX_CASE(12, 2) MTG_DLX_CASE(12, 3) MTG_DLX_CASE(12, 4)
#undef MTG_DLX_CASE
  return hipErrorInvalidValue;
}

}  // namespace mtg
