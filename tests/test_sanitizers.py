"""ASan/UBSan on the host code: the library's host sources (csrc/mtg_host.cpp,
csrc/mtg_host_solve.cpp, csrc/mtg_host_extrema.cpp) and the oracle restatement (oracle/mtg_oracle.c), compiled with
-fsanitize=address,undefined and driven by tests/sanitize/sanitize_driver.cpp.  Host code only: GPU
sanitizers are not available on this pool.  The oracle is test infrastructure; it is compiled here
as the checker the driver compares against."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mav_trajectory_generation_cmake_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_host_code_under_asan_ubsan(tmp_path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)  # the sanitizer runtime must come first in the process
    oracle_o = tmp_path / "oracle.o"
    subprocess.check_call(["gcc", "-std=c99", "-c", "-o", str(oracle_o), os.path.join(ROOT, "oracle", "mtg_oracle.c"),
                           "-I", os.path.join(ROOT, "oracle")] + SAN)
    exe = tmp_path / "sanitize_driver"
    subprocess.check_call(["g++", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                           os.path.join(ROOT, "tests", "sanitize", "sanitize_driver.cpp"),
                           os.path.join(CSRC, "mtg_host.cpp"), os.path.join(CSRC, "mtg_host_solve.cpp"),
                           os.path.join(CSRC, "mtg_host_extrema.cpp"), str(oracle_o),
                           "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-I", os.path.join(ROOT, "oracle"),
                           "-lpthread", "-lm"] + SAN)
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "0 failed checks" in r.stdout


CLANG = "/opt/rocm/llvm/bin"
ARCHER = os.path.join(CLANG, "..", "lib", "libarcher.so")


def _tsan_env():
    env = dict(os.environ, OMP_TOOL_LIBRARIES=ARCHER,
               TSAN_OPTIONS="halt_on_error=1 ignore_noninstrumented_modules=1 exitcode=66")
    env.pop("LD_PRELOAD", None)  # the sanitizer runtime must come first in the process
    return env


def _tsan_build(tmp_path, out, sources, cxx=True):
    cc = os.path.join(CLANG, "clang++" if cxx else "clang")
    subprocess.check_call([cc, "-o", str(out)] + sources + ["-fopenmp", "-fsanitize=thread", "-g", "-O1",
                                                            "-Wl,-rpath," + os.path.join(CLANG, "..", "lib")])


@pytest.mark.skipif(not os.path.exists(ARCHER), reason="needs ROCm clang with libomp + archer")
def test_host_threads_under_tsan(tmp_path):
    """ThreadSanitizer (clang, LLVM libomp with the archer tool so OpenMP synchronisation is seen) over
    every multi-threaded host path: the oracle's OpenMP solve and the product's
    host solve, generators, extrema and vertex maps, each the FIRST call of a fresh process with 8
    threads, then bit-compared with single-threaded runs (tests/sanitize/tsan_driver.cpp).  A
    negative control -- the round-3 race class, a table filled lazily inside the parallel loop
    (tests/sanitize/tsan_negative.c) -- must be reported, or the clean runs prove nothing."""
    neg = tmp_path / "neg"
    _tsan_build(tmp_path, neg, ["-std=c99", os.path.join(ROOT, "tests", "sanitize", "tsan_negative.c")], cxx=False)
    r = subprocess.run([str(neg)], env=_tsan_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 66 and "ThreadSanitizer: data race" in r.stderr, (r.returncode, r.stderr[-2000:])

    oracle_o = tmp_path / "oracle.o"
    subprocess.check_call([os.path.join(CLANG, "clang"), "-std=c99", "-c", "-o", str(oracle_o),
                           os.path.join(ROOT, "oracle", "mtg_oracle.c"), "-I", os.path.join(ROOT, "oracle"),
                           "-fopenmp", "-fsanitize=thread", "-g", "-O1"])
    exe = tmp_path / "tsan_driver"
    _tsan_build(tmp_path, exe, ["-std=c++17", "-ffp-contract=off", os.path.join(ROOT, "tests", "sanitize", "tsan_driver.cpp"),
                                os.path.join(CSRC, "mtg_host.cpp"), os.path.join(CSRC, "mtg_host_solve.cpp"),
                                os.path.join(CSRC, "mtg_host_extrema.cpp"), str(oracle_o),
                                "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-I", os.path.join(ROOT, "oracle"),
                                "-lpthread", "-lm"])
    for first in ("oracle", "host"):
        r = subprocess.run([str(exe), first], env=_tsan_env(), capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, (first, r.stdout[-2000:], r.stderr[-4000:])
        assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
        assert "0 failed checks" in r.stdout


_FRESH = r"""
import sys
import numpy as np
sys.path.insert(0, %r)
from oracle import pyoracle
import mav_trajectory_generation_cmake_amd as mtg
v, m, t = mtg.random_vertices_path_batch(10, 3, 10, 2048, seed0=5, threads=1)
first = %r
if first == "oracle":
    a = pyoracle.solve_linear_batch(10, 4, v, m.astype(np.uint32), t, threads=8, want_cost=True)
    b = pyoracle.solve_linear_batch(10, 4, v, m.astype(np.uint32), t, threads=1, want_cost=True)
    ok = all(np.array_equal(x, y) for x, y in zip(a, b))
else:
    a = mtg.host_solve_linear_batch(10, 4, v, m, t, free=True, cost=True, status=True, threads=8)
    b = mtg.host_solve_linear_batch(10, 4, v, m, t, free=True, cost=True, status=True, threads=1)
    ok = all(np.array_equal(a[k], b[k]) for k in a)
    v8, m8, t8 = mtg.random_vertices_path_batch(10, 3, 10, 2048, seed0=5, threads=8)
    ok = ok and np.array_equal(v8, v) and np.array_equal(m8, m) and np.array_equal(t8, t)
print("BITWISE_OK" if ok else "BITWISE_MISMATCH")
"""


@pytest.mark.parametrize("first", ["oracle", "host"])
def test_fresh_process_first_threaded_call_bitwise(first):
    """The first call of a fresh process is an 8-thread one (the round-3 smoke failure: the oracle's
    table filled lazily inside its OpenMP loop), and must equal the single-threaded run bit for bit."""
    import sys
    r = subprocess.run([sys.executable, "-c", _FRESH % (ROOT, first)], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, MTG_NO_TORCH="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "BITWISE_OK" in r.stdout, r.stdout


def test_host_default_threads_respect_affinity_and_quota():
    """threads <= 0 on the host paths means the CPUs the process may run on (affinity, capped by the
    cgroup CPU quota), not every CPU of the machine (256 on the GPU box against a 16-CPU quota)."""
    from mav_trajectory_generation_cmake_amd import _native as nat
    n = nat.load().mtg_host_default_threads()
    assert 1 <= n <= len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            assert n <= max(1, int(float(q) / float(p)))
    except OSError:
        pass


_CG_DRIVER = r"""
#include "mtg_host_threads.h"
#include <cstdio>
#include <string>
int main(int argc, char** argv) {
  std::string pc;
  for (const char* p = argv[3]; *p; ++p) pc += (*p == ';') ? '\n' : *p;
  std::printf("%d\n", mtg::cgroup_quota_cpus(argv[1], argv[2], pc));
  return 0;
}
"""


def test_cgroup_quota_walks_ancestors_and_v1(tmp_path):
    """mtg::cgroup_quota_cpus: the tightest quota over the process's cgroup and every
    ancestor (a quota on a parent cgroup, or a nested cgroup without a cgroup namespace), and the v1
    cpu.cfs_quota_us / cpu.cfs_period_us files; "max" and -1 mean no quota."""
    src = tmp_path / "cg.cpp"
    src.write_text(_CG_DRIVER)
    exe = tmp_path / "cg"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "mav_trajectory_generation_cmake_amd", "csrc"),
                    str(src), "-o", str(exe)], check=True)
    v2 = tmp_path / "v2"
    v1 = tmp_path / "v1"
    for d, txt in (("", "max 100000"), ("kube", "1600000 100000"), ("kube/pod", "max 100000"),
                   ("kube/pod/ctr", "max 100000"), ("loose", "250000 100000")):
        (v2 / d).mkdir(parents=True, exist_ok=True)
        (v2 / d / "cpu.max").write_text(txt + "\n")
    for d, q, p in (("", -1, 100000), ("a", 800000, 100000), ("a/b", -1, 100000)):
        (v1 / d).mkdir(parents=True, exist_ok=True)
        (v1 / d / "cpu.cfs_quota_us").write_text("%d\n" % q)
        (v1 / d / "cpu.cfs_period_us").write_text("%d\n" % p)

    def run(pc):
        r = subprocess.run([str(exe), str(v2), str(v1), pc], capture_output=True, text=True, check=True)
        return int(r.stdout)
    assert run("0::/kube/pod/ctr") == 16          # the parent's quota caps the nested cgroup
    assert run("0::/loose") == 2                  # its own quota (2.5 CPUs -> 2)
    assert run("0::/") == 0                       # namespace root without a quota
    assert run("12:cpu,cpuacct:/a/b;0::/") == 8   # hybrid: no v2 cpu.max, the v1 quota counts
    assert run("12:cpu,cpuacct:/a/b;0::/loose") == 2  # hybrid with both quotas: the smaller
    assert run("12:cpu,cpuacct:/a/b") == 8        # v1: the ancestor's cfs quota
    assert run("3:memory:/x;5:cpuset:/y") == 0    # no cpu controller line
