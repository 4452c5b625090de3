// mtg_kernels.hip -- hand-written HIP kernels (gfx950) of the batched
// minimum-derivative polynomial optimizer.
//
// What the reference computes per trajectory (lin_impl =
// mav_trajectory_generation/include/mav_trajectory_generation/impl/
// polynomial_optimization_linear_impl.h):
//   Q_i, A_i, A_i^-1           updateSegmentTimes        lin_impl:276-295
//   M (fixed/free reordering)  setupConstraintReorderingMatrix  :172-250
//   R = M^T blkdiag(A^-T Q A^-1) M; R_pp d_p = -R_pf d_f   solveLinear :298-369
//   c_i = A_i^-1 (M d)_i       updateSegmentsFromCompactConstraints :253-273
//   0.5 sum c^T Q c            computeCost               :114-130
//
// How this file computes the same minimiser (DESIGN.md "Algorithm"):
// * Unknowns are ordered by (vertex, derivative), exactly the reference's
//   std::set order (Constraint::operator<, polynomial_optimization_linear.h:273-280),
//   so R is block-tridiagonal with h x h blocks (h = N/2): vertex v couples
//   only to v-1 and v+1.  M is never formed: slot s of segment i is
//   (vertex i + (s >= h), derivative s mod h).
// * Fixed derivatives are eliminated by "pinning": their rows/columns of R
//   become the identity and their values move to the right-hand side, which
//   is algebraically R_pp d_p = -R_pf d_f with uniform h x h blocks for any
//   per-vertex mask (n_free == 0, lin_impl:333-339, falls out naturally).
// * Each block is rebuilt from an exact-rational constant table:
//   H_i = T^(1-2r) S Htilde S,  A_i^-1 = diag(T^-j) A(1)^-1 S,  S = diag(T^(s mod h))
//   (tables from gen_tables.py), which is 3-6 orders more accurate than
//   forming A^-1 and A^-T Q A^-1 in FP64.
// * The block-tridiagonal SPD system is solved by block Thomas elimination
//   with h x h Cholesky factors: S_v = D_v - E_{v-1}^T G_{v-1},
//   [G_v | z_v] = S_v^-1 [E_v | rhs_v], back: x_v = z_v - G_v x_{v+1}.
//
// Mapping to CDNA4: a trajectory is owned by a group of LG lanes (LG = 8 for
// N=10, D=3, so 8 trajectories per wave64).  Lane c < h owns column c of
// [E_v | G_v]; lane h + d owns dimension d's right-hand side.  Per vertex every
// lane forms its column with four h x h (or h x N) mat-vecs against Htilde held
// in the scalar cache, the h columns of S_v are exchanged through LDS, every
// lane factors the h x h S_v redundantly in registers (SIMD: redundancy is
// free), and solves its own column.  G_v and z_v stay in LDS for the backward
// sweep, which also recovers coefficients and the cost and streams them to HBM.
// Everything is FP64 (the reference is FP64 throughout).
#include "mtg_device.h"
#include "mtg_fused.inc"

#include <stdlib.h>

namespace mtg {

template <int N, int R>
__global__ __launch_bounds__(kBlock) void solve_fused_kernel(SolveArgs a, int lg_log2) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  solve_fused_block<N, R>(a, lg_log2, (int64_t)blockIdx.x * (kBlock >> lg_log2), lds);
}

bool solve_geometry(int N, int D, int K, int* lanes_per_traj, size_t* lds_bytes, int* traj_per_block) {
  const int H = N / 2;
  const int need = H + D;
  int lg = 8;
  while (lg < need) lg *= 2;
  if (lg > 64) return false;
  for (;;) {
    const size_t bytes = (size_t)(kBlock / lg) * slot_doubles(H, D, K, lg) * sizeof(double);
    if (bytes <= kMaxLdsPerBlock || (lg == 64 && bytes <= kMaxLdsHard)) {
      *lanes_per_traj = lg;
      *lds_bytes = bytes;
      *traj_per_block = kBlock / lg;
      return true;
    }
    if (lg == 64) return false;
    lg *= 2;
  }
}

template <int N, int R>
static hipError_t launch_fused_nr(const SolveArgs& a, hipStream_t stream) {
  int lg, tpb;
  size_t lds;
  if (!solve_geometry(N, a.D, a.K, &lg, &lds, &tpb)) return hipErrorInvalidValue;
  int lg_log2 = 0;
  while ((1 << lg_log2) < lg) ++lg_log2;
  const int64_t blocks = (a.B + tpb - 1) / tpb;
  if (blocks == 0) return hipSuccess;
  static const size_t lds_pad = [] {  // occupancy experiments only (DESIGN.md "Occupancy")
    const char* p = getenv("MTG_DEBUG_LDS_PAD");
    return p ? (size_t)atoi(p) : (size_t)0;
  }();
  lds += lds_pad;
  if (lds > kMaxLdsPerBlock) {
    hipError_t e = hipFuncSetAttribute((const void*)solve_fused_kernel<N, R>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  launch_kernel((solve_fused_kernel<N, R>), dim3((unsigned)blocks), dim3(kBlock), lds, stream, a, lg_log2);
  return hipGetLastError();
}

template <int N>
static hipError_t launch_fused_n(const SolveArgs& a, hipStream_t stream) {
  switch (a.r) {
    case 0: return launch_fused_nr<N, 0>(a, stream);
    case 1: if constexpr (N / 2 > 1) return launch_fused_nr<N, 1>(a, stream); break;
    case 2: if constexpr (N / 2 > 2) return launch_fused_nr<N, 2>(a, stream); break;
    case 3: if constexpr (N / 2 > 3) return launch_fused_nr<N, 3>(a, stream); break;
    case 4: if constexpr (N / 2 > 4) return launch_fused_nr<N, 4>(a, stream); break;
    case 5: if constexpr (N / 2 > 5) return launch_fused_nr<N, 5>(a, stream); break;
    default: break;
  }
  return hipErrorInvalidValue;
}

int solve_kernel(int N, int D, int K, unsigned flags, int r, int64_t B) {
  int lg;
  size_t lds;
  if (flags & MTG_FLAG_GENERAL_KERNEL) return MTG_KERNEL_GENERAL;
  // the dimension-lane kernel wherever it applies, at every batch size, so that a
  // trajectory's result does not depend on the size of the call it is in; MTG_FLAG_COLUMN_KERNEL
  // keeps the column kernel (A/B)
  const bool dl_default = !(flags & MTG_FLAG_COLUMN_KERNEL);
  if (((flags & MTG_FLAG_DL_KERNEL) || dl_default) && r >= 0 && dl_geometry(N, D, K, r)) return MTG_KERNEL_DL;
  if (reg_geometry(N, D, K, &lg, &lds)) return MTG_KERNEL_COLUMN;
  // chains of other lengths: the long-chain dimension-lane kernel (with the general kernel's block
  // function for the trajectories it does not serve)
  if (((flags & MTG_FLAG_DL_KERNEL) || dl_default) && r >= 0 && dlx_geometry(N, D, K, r)) return MTG_KERNEL_DLX;
  return MTG_KERNEL_GENERAL;
}

hipError_t launch_solve(int N, const SolveArgs& a, hipStream_t stream, unsigned flags) {
  switch (solve_kernel(N, a.D, a.K, flags, a.r, a.B)) {
    case MTG_KERNEL_DL: return launch_solve_dl(N, a, stream);
    case MTG_KERNEL_COLUMN: return launch_solve_reg(N, a, stream);
    case MTG_KERNEL_DLX: return launch_solve_dlx(N, a, stream);  // (a.work: the caller's)
    default: break;
  }
  switch (N) {
    case 2: return launch_fused_n<2>(a, stream);
    case 4: return launch_fused_n<4>(a, stream);
    case 6: return launch_fused_n<6>(a, stream);
    case 8: return launch_fused_n<8>(a, stream);
    case 10: return launch_fused_n<10>(a, stream);
    case 12: return launch_fused_n<12>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
