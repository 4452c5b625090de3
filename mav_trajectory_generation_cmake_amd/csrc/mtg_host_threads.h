// Default worker count of the host paths (generators, host solve, host extrema) when the caller
// passes threads <= 0: the CPUs this process may actually run on -- the affinity mask, capped by
// the tightest CPU quota of its cgroup and every ancestor (cgroup v2 cpu.max; cgroup v1
// cpu.cfs_quota_us / cpu.cfs_period_us) -- not std::thread::hardware_concurrency(), which counts
// every CPU of the machine (256 on the MI355X box against a 16-CPU quota: 16x oversubscribed).
// Plain C++ (no HIP): the host sources are also built on their own for the sanitizer runs.
#pragma once

#include <sched.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

namespace mtg {

// CPUs allowed by the quota file(s) of one cgroup directory, or 0 for none (no file, "max", -1)
inline int cgroup_dir_cpus(const std::string& dir, bool v2) {
  long long quota = 0, period = 0;
  if (v2) {
    FILE* f = std::fopen((dir + "/cpu.max").c_str(), "r");
    if (!f) return 0;
    char q[32] = {0};
    const bool ok = std::fscanf(f, "%31s %lld", q, &period) == 2 && period > 0 && q[0] != 'm' &&
                    std::sscanf(q, "%lld", &quota) == 1;
    std::fclose(f);
    if (!ok) return 0;
  } else {
    FILE* fq = std::fopen((dir + "/cpu.cfs_quota_us").c_str(), "r");
    FILE* fp = std::fopen((dir + "/cpu.cfs_period_us").c_str(), "r");
    const bool ok = fq && fp && std::fscanf(fq, "%lld", &quota) == 1 && std::fscanf(fp, "%lld", &period) == 1;
    if (fq) std::fclose(fq);
    if (fp) std::fclose(fp);
    if (!ok || period <= 0) return 0;
  }
  if (quota <= 0) return 0;
  return quota / period > 0 ? (int)(quota / period) : 1;
}

// The tightest quota over the process's cgroup and its ancestors.  root_v2: where the unified
// hierarchy is mounted (/sys/fs/cgroup); root_v1: the v1 cpu controller's directory; proc_cgroup: the
// contents of /proc/self/cgroup ("0::/path" for v2, "N:cpu,cpuacct:/path" for v1).  A hybrid host
// (systemd's hybrid mode) has both lines: the v2 walk finds no cpu.max there (the controller is in
// the v1 tree), so both hierarchies are walked and the smaller quota is taken.  Without a cgroup
// namespace the path is the full one and the walk visits every ancestor; inside one (the path is
// "/") it reads the namespace root, which is the container's own quota.  0: no quota found.
inline int cgroup_walk_cpus(const std::string& root, std::string path, bool v2) {
  int best = 0;
  for (;;) {  // this cgroup, then each ancestor up to the mount root
    const int c = cgroup_dir_cpus(root + (path == "/" ? "" : path), v2);
    if (c > 0 && (best == 0 || c < best)) best = c;
    if (path.empty() || path == "/") break;
    const size_t s = path.find_last_of('/');
    path = s == 0 || s == std::string::npos ? "/" : path.substr(0, s);
  }
  return best;
}

inline int cgroup_quota_cpus(const std::string& root_v2, const std::string& root_v1, const std::string& proc_cgroup) {
  std::string p2, p1;
  bool has2 = false, has1 = false;
  size_t pos = 0;
  while (pos < proc_cgroup.size()) {
    size_t end = proc_cgroup.find('\n', pos);
    if (end == std::string::npos) end = proc_cgroup.size();
    const std::string line = proc_cgroup.substr(pos, end - pos);
    pos = end + 1;
    const size_t c1 = line.find(':'), c2 = c1 == std::string::npos ? c1 : line.find(':', c1 + 1);
    if (c2 == std::string::npos) continue;
    const std::string ctrl = line.substr(c1 + 1, c2 - c1 - 1);
    if (line.compare(0, c1, "0") == 0 && ctrl.empty()) {  // v2 unified hierarchy
      p2 = line.substr(c2 + 1);
      has2 = true;
    } else {  // v1: the line naming the cpu controller
      size_t p = 0;
      while (p <= ctrl.size()) {
        size_t q = ctrl.find(',', p);
        if (q == std::string::npos) q = ctrl.size();
        if (ctrl.compare(p, q - p, "cpu") == 0) {
          p1 = line.substr(c2 + 1);
          has1 = true;
        }
        p = q + 1;
      }
    }
  }
  if (!has2 && !has1) return cgroup_walk_cpus(root_v2, "/", true);
  const int c2 = has2 ? cgroup_walk_cpus(root_v2, p2, true) : 0;
  const int c1 = has1 ? cgroup_walk_cpus(root_v1, p1, false) : 0;
  return c2 > 0 && (c1 == 0 || c2 < c1) ? c2 : c1;
}

inline int usable_cpus_uncached() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) {
    const int a = CPU_COUNT(&set);
    if (a > 0 && (n <= 0 || a < n)) n = a;
  }
  std::string pc;
  if (FILE* f = std::fopen("/proc/self/cgroup", "r")) {
    char buf[512];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof(buf), f)) > 0) pc.append(buf, k);
    std::fclose(f);
  }
  const int c = cgroup_quota_cpus("/sys/fs/cgroup", "/sys/fs/cgroup/cpu", pc);
  if (c > 0 && (n <= 0 || c < n)) n = c;
  return n > 0 ? n : 1;
}

// computed once per process (a function-local static: initialisation is thread-safe)
inline int usable_cpus() {
  static const int n = usable_cpus_uncached();
  return n;
}

}  // namespace mtg
