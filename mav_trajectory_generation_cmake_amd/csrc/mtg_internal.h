// Internal declarations shared by the kernels (mtg_kernels.hip) and the C ABI
// (mtg_capi.hip).  Not installed; the public surface is include/mtg.h.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtg.h"

namespace mtg {

// Timing events for the next kernel launch, set by the C ABI around a timed call: launch_kernel()
// records them in the kernel's own dispatch packet (hipExtLaunchKernelGGL) instead of as two
// separate marker packets in the stream.
struct PendingEvents {
  hipEvent_t start = nullptr, stop = nullptr;
  bool used = false;
};
PendingEvents& pending_events();  // per host thread

template <typename F, typename... Args>
inline void launch_kernel(F kernel, const dim3& grid, const dim3& block, uint32_t lds, hipStream_t stream,
                          Args... args) {
  PendingEvents& pe = pending_events();
  if (pe.start && !pe.used) {
    pe.used = true;
    hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, pe.start, pe.stop, 0u, args...);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, lds, stream, args...);
  }
}

// Arguments of one batched solve launch.  Pointers are device pointers.
struct SolveArgs {
  const double* values;   // [B][V][h][D]
  const uint8_t* mask;    // [B][V]
  const double* times;    // [B][K]
  double* coeffs;         // [B][K][D][N]
  double* free_out;       // [B][D][V*h]  (nullable)
  int32_t* n_free_out;    // [B]          (nullable)
  double* cost_out;       // [B]          (nullable)
  int32_t* status;        // [B]          (nullable)
  const double* scales;   // time-sweep candidate scales [C] (nullable: plain solve)
  int64_t B;              // trajectories (or trajectory x candidate pairs for the sweep)
  int K, D, r;
  int n_cand;             // candidates per trajectory for the sweep (1 for a plain solve)
  int gi;                 // register column kernel: G in LDS for the interior-waypoint body (set by
                          // launch_solve_reg, mtg_solve_reg.inc reg_gi_doubles)
  double* work;           // long-chain dimension-lane kernel: its workspace (dlx_workspace_bytes)
  int64_t work_bytes;
};

// Lanes per trajectory and LDS bytes per workgroup for a shape; returns false
// when the per-trajectory working set cannot fit in LDS.
bool solve_geometry(int N, int D, int K, int* lanes_per_traj, size_t* lds_bytes, int* traj_per_block);

// Launch the fused solve on `stream` with the kernel solve_kernel() picks: the register column
// kernel (mtg_solve_reg.hip) where reg_geometry allows it (K <= 12, or N = 12 with K <= 20), else
// the general LDS-resident kernel (mtg_kernels.hip); the dimension-lane kernel (mtg_solve_dl.hip)
// where dl_geometry allows it; MTG_FLAG_GENERAL_KERNEL the general kernel.
// B: the batch (trajectories, or trajectory x candidate pairs; < 0: unknown).  The choice does not
// depend on it (since round 4: the DL kernel at every size where it applies).
int solve_kernel(int N, int D, int K, unsigned flags, int r = -1, int64_t B = -1);  // MTG_KERNEL_*
hipError_t launch_solve(int N, const SolveArgs& a, hipStream_t stream, unsigned flags = 0);
bool reg_geometry(int N, int D, int K, int* lanes_per_traj, size_t* lds_bytes);
hipError_t launch_solve_reg(int N, const SolveArgs& a, hipStream_t stream);
// dimension-lane kernel of the interior-waypoint pattern (mtg_solve_dl.hip: ends fix every
// derivative, interior vertices exactly their position): one lane per (chain, dimension)
bool dl_geometry(int N, int D, int K, int r);
hipError_t launch_solve_dl(int N, const SolveArgs& a, hipStream_t stream);
// the same recurrence for chains of any length (mtg_solve_dlx.hip), where neither the DL kernel nor
// the column kernel applies; its workspace (a.work) holds dlx_workspace_bytes for the launch's batch
bool dlx_geometry(int N, int D, int K, int r);
size_t dlx_workspace_bytes(int N, int D, int K, int64_t B);
hipError_t launch_solve_dlx(int N, const SolveArgs& a, hipStream_t stream);

// Two-kernel path (MTG_FLAG_SPLIT_KERNELS): assembly into the block-tridiagonal
// workspace, then the block-Cholesky solve + recovery.
size_t split_workspace_bytes(int N, int D, int K, int64_t B);
hipError_t launch_solve_split(int N, const SolveArgs& a, void* workspace, hipStream_t stream);

// cost / gradient of fixed vertex derivatives at candidate times (mtg_cost.hip)
size_t cost_lds_bytes(int N, int D, int K);
hipError_t launch_cost_at_times(int N, int r, const double* values, const uint8_t* mask, const double* times,
                                const double* scales, double* cost, double* grad, int64_t B, int K, int D, int C,
                                hipStream_t stream);

// segment-time cost sweep + time Jacobian on the matrix cores (mtg_jacobian.hip)
size_t time_jacobian_lds_bytes(int N, int D, int K, int C);
hipError_t launch_time_jacobian(int N, int r, const double* values, const double* times, const double* scales,
                                double* cost, double* jac, double delta, int64_t B, int K, int D, int C,
                                hipStream_t stream);

// vertex derivatives <-> coefficients (mtg_vertex.hip)
bool vertex_map_fits(int N, int D, int K);
hipError_t launch_vertex_map(bool to_coeffs, int N, const double* in, const double* times, double* out, int64_t B,
                             int K, int D, hipStream_t stream);

// min / max magnitude of a derivative over trajectories (mtg_extrema.hip)
hipError_t launch_min_max_magnitude(int N, const double* coeffs, const double* times, int64_t B, int K, int D,
                                    int derivative, unsigned dims, mtg_extremum* mn, mtg_extremum* mx,
                                    hipStream_t stream);

// evaluateRange
hipError_t launch_eval_count(int N, int D, int K, int64_t B, const double* times, double t_start,
                             double t_end, double dt, int64_t* counts, hipStream_t stream);
// run-table workspace of launch_eval_range (bytes; *cap = runs stored per trajectory)
size_t eval_workspace_bytes(int K, int64_t B, int* cap);
// Samples of every trajectory (one block each).  Without runs_ready the run table is built first
// (eval_runs_kernel); with runs_ready, launch_eval_runs_counts already built it together with the
// counts and the two-level offsets: offsets then holds the in-block prefix and the kernel writes the
// final offsets to offsets_out.  A trajectory whose samples would end past `capacity` samples is
// not written, and none is when the device-side `total` (nullable) exceeds it.
hipError_t launch_eval_range(int N, int D, int K, int64_t B, const double* coeffs,
                             const double* times, double t_start, double t_end, double dt,
                             int derivative, const int64_t* counts, const int64_t* offsets, double* out,
                             double* sample_times, void* ws, int cap, hipStream_t stream, bool runs_ready = false,
                             int64_t* offsets_out = nullptr, int64_t capacity = INT64_MAX,
                             const int64_t* total = nullptr);
// The one-call evaluateRange's first two kernels: the run table plus counts[B] and the in-block
// offsets (eval_runs_kernel), then the block offsets and the grand total (eval_scan_kernel); all
// device-side, no host round trip.  Workspace: eval_full_workspace_bytes.
size_t eval_full_workspace_bytes(int K, int64_t B, int* cap);
hipError_t launch_eval_runs_counts(int K, int64_t B, const double* times, double t_start, double t_end, double dt,
                                   int64_t* counts, int64_t* offsets, void* ws, int cap, int64_t* total,
                                   hipStream_t stream);

}  // namespace mtg
