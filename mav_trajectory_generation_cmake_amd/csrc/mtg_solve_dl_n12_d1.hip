// One (N, D) of the dimension-lane kernel (mtg_solve_dl.inc).
#include "mtg_solve_dl.inc"

namespace mtg {
MTG_DL_LAUNCHER(12, 1)
}  // namespace mtg
