// One (N, D) of the long-chain dimension-lane kernel (mtg_solve_dlx.inc).
#include "mtg_solve_dlx.inc"

namespace mtg {
MTG_DLX_LAUNCHER(8, 1)
}  // namespace mtg
