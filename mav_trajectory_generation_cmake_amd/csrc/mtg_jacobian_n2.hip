// One N of the matrix-core segment-time sweep (mtg_jacobian.inc).
#include "mtg_jacobian.inc"

namespace mtg {
MTG_JAC_LAUNCHER(2)
}  // namespace mtg
