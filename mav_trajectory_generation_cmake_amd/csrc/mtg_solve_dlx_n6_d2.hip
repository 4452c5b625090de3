// One (N, D) of the long-chain dimension-lane kernel (mtg_solve_dlx.inc).
#include "mtg_solve_dlx.inc"

namespace mtg {
MTG_DLX_LAUNCHER(6, 2)
}  // namespace mtg
