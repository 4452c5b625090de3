// runtime.h -- how the drop-in classes reach the library (libmav_trajectory_generation.so, C ABI
// include/mtg.h): error behaviour, the process-wide GPU context, and where single problems run.
//
// Error behaviour.  The reference CHECK-fails (glog: prints and aborts) on a bad
// derivative_to_optimize (lin_impl:50-55), mismatched sizes (:66-67), non-positive segment times
// (:287) and null out-parameters.  So does this API, unless MTG_CPP_THROW is defined, in which case
// it throws mav_trajectory_generation::Error (the C++ tests use that).  Invalid constraint orders
// are dropped with a warning on stderr (LOG(WARNING), lin_impl:82-87).
//
// Execution policy.  One problem (PolynomialOptimization<N>::solveLinear, BASELINE config 1) is a
// few microseconds of arithmetic; a GPU round trip costs ~40 us.  By default (kAuto) single
// problems therefore run on the library's host solver (mtg_host_solve_linear_batch, the same
// algorithm as the HIP kernels) and batches (BatchPolynomialOptimization<N>) on the GPU.
// kDevice sends single problems through the GPU too; kHost keeps everything on the CPU.  The
// environment variable MTG_EXECUTION=auto|host|device sets the initial policy.
#ifndef MAV_TRAJECTORY_GENERATION_RUNTIME_H_
#define MAV_TRAJECTORY_GENERATION_RUNTIME_H_

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

#include "mtg.h"

namespace mav_trajectory_generation {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

[[noreturn]] inline void fail(int code, const std::string& what) {
#ifdef MTG_CPP_THROW
  throw Error(code, what);
#else
  std::fprintf(stderr, "mav_trajectory_generation: check failed: %s (%s)\n", what.c_str(), mtg_status_string(code));
  std::abort();
#endif
}

inline void warn(const std::string& what) { std::fprintf(stderr, "mav_trajectory_generation: warning: %s\n", what.c_str()); }

inline void check(int rc, mtg_ctx* ctx, const char* where) {
  if (rc != MTG_OK) {
    std::string msg = where;
    const char* detail = ctx ? mtg_last_error(ctx) : nullptr;
    if (detail && *detail) msg += std::string(": ") + detail;
    fail(rc, msg);
  }
}

// CHECK_NOTNULL
template <typename T>
inline T* check_notnull(T* p, const char* what) {
  if (!p) fail(MTG_ERR_INVALID_ARGUMENT, std::string(what) + " must not be null");
  return p;
}

enum class ExecutionPolicy { kAuto = 0, kHost = 1, kDevice = 2 };

namespace detail {
inline std::atomic<int>& policy_slot() {
  static std::atomic<int> p([] {
    const char* e = std::getenv("MTG_EXECUTION");
    if (e && !std::strcmp(e, "host")) return (int)ExecutionPolicy::kHost;
    if (e && !std::strcmp(e, "device")) return (int)ExecutionPolicy::kDevice;
    return (int)ExecutionPolicy::kAuto;
  }());
  return p;
}
}  // namespace detail

inline void setExecutionPolicy(ExecutionPolicy p) { detail::policy_slot().store((int)p); }
inline ExecutionPolicy getExecutionPolicy() { return (ExecutionPolicy)detail::policy_slot().load(); }
// single-problem calls go to the GPU only under kDevice
inline bool singleOnDevice() { return getExecutionPolicy() == ExecutionPolicy::kDevice; }

// One process-wide context on device 0 for single-problem GPU calls (created on first use).
inline mtg_ctx* defaultContext() {
  static std::once_flag once;
  static mtg_ctx* ctx = nullptr;
  std::call_once(once, [] { check(mtg_create(0, &ctx), nullptr, "mtg_create(0)"); });
  return ctx;
}

}  // namespace mav_trajectory_generation

#endif  // MAV_TRAJECTORY_GENERATION_RUNTIME_H_
