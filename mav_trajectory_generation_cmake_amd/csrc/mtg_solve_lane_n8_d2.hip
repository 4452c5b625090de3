// One (N, D) of the lane-per-chain solve kernel (mtg_solve_lane.inc).
#include "mtg_solve_lane.inc"

namespace mtg {
MTG_LANE_LAUNCHER(8, 2)
}  // namespace mtg
