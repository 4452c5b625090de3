// The wide register-resident bucket, N = 12, 12 < K <= 20, r = 0 (mtg_solve_reg.inc).
#include "mtg_solve_reg.inc"

namespace mtg {
MTG_REG_WIDE_LAUNCHER(0)
}  // namespace mtg
