// mtg_solve_reg.hip -- dispatch of the register-resident solve kernel (mtg_solve_reg.inc; one
// translation unit per N in mtg_solve_reg_n*.hip).
#include "mtg_solve_reg.inc"  // (templates only: no kernel is instantiated in this unit)

namespace mtg {

hipError_t launch_solve_reg_n2(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n4(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n6(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n8(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n10(const SolveArgs&, int, size_t, hipStream_t);
hipError_t launch_solve_reg_n12(const SolveArgs&, int, size_t, hipStream_t);


bool reg_geometry(int N, int D, int K, int* lanes_per_traj, size_t* lds_bytes) {
  const int H = N / 2;
  // G_v columns take H * KMAX doubles per lane: beyond ~50 the 2-waves-per-SIMD kernel spills
  // (N=12, K > 8); the wide bucket (N = 12, K <= 20) keeps G in LDS instead (Forward::GLDS)
  const int km = reg_kmax(K);
  if (km < 0 || (H * km > 50 && !(N == 12 && km == kRegKMaxWide))) return false;
  int lc = 8;  // lanes per chain: h column lanes + D dimension lanes
  while (lc < H + D) lc *= 2;
  const int lg = kTwist ? 2 * lc : lc;  // twisted: two chains per trajectory
  if (lg > 64) return false;
  const size_t bytes = (size_t)reg_lds_doubles(N, D, K, lg, kTwist) * sizeof(double);
  if (bytes > kMaxLdsPerBlock) return false;
  *lanes_per_traj = lg;
  *lds_bytes = bytes;
  return true;
}

// G in LDS for the interior-waypoint body (reg_gi_doubles) shortens each wave's backward sweep but
// takes LDS (config 2: 10.8 -> 15.0 KB per wave): use it when every wave of the launch is resident
// at once under the larger footprint (config 2 at B = 1e4: 18.5 -> 17.7 us), not when the launch
// runs in rounds (B = 131072: 157 -> 161 us, 12 -> 10 waves per CU).
static bool use_gi(int N, const SolveArgs& a, int lg, size_t lds_plain, size_t* lds_gi) {
  if (!kTwist || reg_gi_doubles(N, a.K, kTwist) == 0) return false;
  const size_t bytes = (size_t)reg_lds_doubles(N, a.D, a.K, lg, kTwist, true) * sizeof(double);
  if (bytes > kMaxLdsPerBlock) return false;
  *lds_gi = bytes;
  if (bytes == lds_plain) return true;  // (the G block fits the epilogue's staging area: free)
  // the device's CU count and LDS per CU, cached per thread for its current device
  thread_local int dev_cached = -1, cus = 0, lds_cu = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (dev != dev_cached) {
    int c = 0, l = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipDeviceGetAttribute(&l, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess)
      return false;
    dev_cached = dev;
    cus = c;
    lds_cu = l;
  }
  if (cus <= 0 || lds_cu <= 0) return false;
  const int64_t tpb = kBlock / lg, waves = (a.B + tpb - 1) / tpb;
  const size_t alloc = (bytes + 511) & ~(size_t)511;  // (LDS allocation granule)
  int64_t per_cu = (int64_t)(lds_cu / alloc);
  if (per_cu > 4 * MTG_REG_WAVES) per_cu = 4 * MTG_REG_WAVES;
  return waves <= per_cu * cus;
}

hipError_t launch_solve_reg(int N, const SolveArgs& a0, hipStream_t stream) {
  int lg;
  size_t lds;
  if (!reg_geometry(N, a0.D, a0.K, &lg, &lds)) return hipErrorInvalidValue;
  SolveArgs a = a0;
  a.gi = 0;
  size_t lds_gi = 0;
  if (use_gi(N, a, lg, lds, &lds_gi)) {
    a.gi = 1;
    lds = lds_gi;
  }
  switch (N) {
    case 2: return launch_solve_reg_n2(a, lg, lds, stream);
    case 4: return launch_solve_reg_n4(a, lg, lds, stream);
    case 6: return launch_solve_reg_n6(a, lg, lds, stream);
    case 8: return launch_solve_reg_n8(a, lg, lds, stream);
    case 10: return launch_solve_reg_n10(a, lg, lds, stream);
    case 12: return launch_solve_reg_n12(a, lg, lds, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
