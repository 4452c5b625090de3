// One N of the register-resident solve kernel (mtg_solve_reg.inc).
#include "mtg_solve_reg.inc"

namespace mtg {
MTG_REG_LAUNCHER(6)
}  // namespace mtg
