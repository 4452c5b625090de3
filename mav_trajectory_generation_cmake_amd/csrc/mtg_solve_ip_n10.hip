// One N of the interior-waypoint lane kernel (mtg_solve_ip.inc), D = 1..4.
#include "mtg_solve_ip.inc"

namespace mtg {
MTG_IP_LAUNCHER(10)
}  // namespace mtg
