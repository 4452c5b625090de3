// The wide register-resident bucket, N = 12, 12 < K <= 20, r = 2 (mtg_solve_reg.inc).
#include "mtg_solve_reg.inc"

namespace mtg {
MTG_REG_WIDE_LAUNCHER(2)
}  // namespace mtg
