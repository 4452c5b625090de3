// mtg_jacobian.hip -- dispatch of the matrix-core segment-time sweep (mtg_jacobian.inc; one
// translation unit per N in mtg_jacobian_n*.hip).
#include "mtg_jacobian.inc"  // (templates only: no kernel is instantiated in this unit)

namespace mtg {

hipError_t launch_time_jacobian_n2(const JacArgs&, int, hipStream_t);
hipError_t launch_time_jacobian_n4(const JacArgs&, int, hipStream_t);
hipError_t launch_time_jacobian_n6(const JacArgs&, int, hipStream_t);
hipError_t launch_time_jacobian_n8(const JacArgs&, int, hipStream_t);
hipError_t launch_time_jacobian_n10(const JacArgs&, int, hipStream_t);
hipError_t launch_time_jacobian_n12(const JacArgs&, int, hipStream_t);

size_t time_jacobian_lds_bytes(int N, int D, int K, int C) { return sizeof(double) * jac_lds_doubles(N, D, K, C); }

hipError_t launch_time_jacobian(int N, int r, const double* values, const double* times, const double* scales,
                                double* cost, double* jac, double delta, int64_t B, int K, int D, int C,
                                hipStream_t stream) {
  JacArgs a{values, times, scales, cost, jac, delta, B, K, D, C};
  switch (N) {
    case 2: return launch_time_jacobian_n2(a, r, stream);
    case 4: return launch_time_jacobian_n4(a, r, stream);
    case 6: return launch_time_jacobian_n6(a, r, stream);
    case 8: return launch_time_jacobian_n8(a, r, stream);
    case 10: return launch_time_jacobian_n10(a, r, stream);
    case 12: return launch_time_jacobian_n12(a, r, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mtg
