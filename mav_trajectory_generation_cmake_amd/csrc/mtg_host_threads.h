// Default worker count of the host paths (generators, host solve, host extrema) when the caller
// passes threads <= 0: the CPUs this process may actually run on -- the affinity mask, capped by
// the cgroup v2 CPU quota (cpu.max) -- not std::thread::hardware_concurrency(), which counts every
// CPU of the machine (256 on the MI355X box against a 16-CPU quota: 16x oversubscribed).
// Plain C++ (no HIP): the host sources are also built on their own for the sanitizer runs.
#pragma once

#include <sched.h>

#include <cstdio>
#include <thread>

namespace mtg {

inline int usable_cpus_uncached() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) {
    const int a = CPU_COUNT(&set);
    if (a > 0 && (n <= 0 || a < n)) n = a;
  }
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    if (std::fscanf(f, "%31s %lld", q, &period) == 2 && period > 0 && q[0] != 'm') {
      long long quota = 0;
      if (std::sscanf(q, "%lld", &quota) == 1 && quota > 0) {
        const int c = (int)(quota / period) > 0 ? (int)(quota / period) : 1;
        if (n <= 0 || c < n) n = c;
      }
    }
    std::fclose(f);
  }
  return n > 0 ? n : 1;
}

// computed once per process (a function-local static: initialisation is thread-safe)
inline int usable_cpus() {
  static const int n = usable_cpus_uncached();
  return n;
}

}  // namespace mtg
