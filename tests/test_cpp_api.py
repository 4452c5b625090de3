"""The C++ drop-in (include/mav_trajectory_generation/*.h over libmav_trajectory_generation.so).

CPU: the CMake project builds the `mav_trajectory_generation` target (the reference's target name,
mav_trajectory_generation/CMakeLists.txt:46) and the C++ API test against the drop-in headers; the
test runs its host-solver half, and the matrices the drop-in exposes (getA / getAInverse / getM /
getR / getMpinv, polynomial_optimization_linear.h:209-214) are compared with the oracle's.
GPU: the same C++ test with single problems sent through the GPU, plus the batched API."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from mav_trajectory_generation_cmake_amd import _native as nat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_cpp_api.cpp")
BUILD = os.path.join(ROOT, "build")


def _cmake_build():
    """Configure (once) and build the project's default targets, the library and test_cpp_api,
    incrementally in build/ (the tree __graft_entry__.build() uses)."""
    cmake = shutil.which("cmake")
    if cmake is None:
        pytest.skip("cmake not available")
    if not os.path.exists(os.path.join(BUILD, "CMakeCache.txt")):
        subprocess.run([cmake, "-S", ROOT, "-B", BUILD, "-DCMAKE_BUILD_TYPE=Release"], check=True,
                       capture_output=True)
    r = subprocess.run([cmake, "--build", BUILD, "-j", str(min(8, os.cpu_count() or 1))], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    exe = os.path.join(BUILD, "test_cpp_api")
    assert os.path.exists(exe)
    return exe


def _gxx_build(tmp_path):
    cxx = shutil.which("g++") or "g++"
    exe = tmp_path / "test_cpp_api"
    libdir = os.path.dirname(nat.LIB_PATH)
    subprocess.run([cxx, "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-DMTG_CPP_THROW=1", "-I",
                    os.path.join(ROOT, "include"), SRC, "-o", str(exe), "-L", libdir, "-lmav_trajectory_generation",
                    "-Wl,-rpath," + libdir], check=True)
    return str(exe)


def test_cmake_builds_drop_in_and_host_checks_pass():
    exe = _cmake_build()
    r = subprocess.run([exe, "host"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def _read_dump(path):
    raw = np.fromfile(path, dtype=np.float64)
    out, i = [], 0
    while i < len(raw):
        r, c = int(raw[i]), int(raw[i + 1])
        out.append(raw[i + 2:i + 2 + r * c].reshape(r, c))
        i += 2 + r * c
    return out


def _blkdiag(blocks):
    K, N, _ = blocks.shape
    out = np.zeros((K * N, K * N))
    for i in range(K):
        out[i * N:(i + 1) * N, i * N:(i + 1) * N] = blocks[i]
    return out


def test_drop_in_matrices_match_oracle(tmp_path):
    """getA / getAInverse / getM / getR / getMpinv / getFixedConstraints / getFreeConstraints /
    computeCost of one problem (createRandomVertices(SNAP, 5, [-10,-20,-10], [10,20,10], 12345) plus a
    fixed velocity at vertex 2, estimateSegmentTimes(3, 5)) against the oracle's restatement of
    lin_impl (its M, A, Schur A^-1, Q, R = M^T A^-T Q A^-1 M, QR solve)."""
    from oracle import pyoracle as O
    exe = _cmake_build()
    path = str(tmp_path / "mats.bin")
    subprocess.run([exe, "dump", path], check=True, timeout=120)
    A, Ai, M, R, Mp, fx, fr, tm, cost = _read_dump(path)
    N, r = 10, 4
    vals, mask = O.create_random_vertices(4, 5, [-10, -20, -10], [10, 20, 10], 12345, nd=5)
    vals[2, 1, :] = [0.5, -0.25, 1.0]
    mask[2] |= 2
    times = O.estimate_segment_times(vals, 3.0, 5.0)
    np.testing.assert_allclose(tm[0], times, rtol=1e-15, atol=0)
    ref = O.solve_linear(N, r, vals, mask, times, want_matrices=True)
    K = len(times)
    # A: the same formula (setupMappingMatrix) -> identical
    np.testing.assert_array_equal(A, _blkdiag(ref["amap"]))
    # A^-1: exact table scaled by T vs the reference's FP64 Schur inverse
    Ai_ref = _blkdiag(ref["ainv"])
    assert np.max(np.abs(Ai - Ai_ref) / np.maximum(np.abs(Ai_ref), 1e-300)) < 1e-12
    # M: exactly the reference's 0/1 reordering matrix
    M_ref = np.zeros_like(M)
    M_ref[np.arange(len(ref["col_of_row"])), ref["col_of_row"]] = 1.0
    np.testing.assert_array_equal(M, M_ref)
    Mp_ref = M_ref.T / M_ref.T.sum(axis=1, keepdims=True)
    np.testing.assert_array_equal(Mp, Mp_ref)
    # R = M^T blkdiag(A^-T Q A^-1) M
    H = np.stack([ref["ainv"][i].T @ ref["qmat"][i] @ ref["ainv"][i] for i in range(K)])
    R_ref = M_ref.T @ _blkdiag(H) @ M_ref
    scale = np.sqrt(np.outer(np.abs(np.diag(R_ref)), np.abs(np.diag(R_ref))))
    assert np.max(np.abs(R - R_ref) / scale) < 1e-9
    np.testing.assert_array_equal(fx, ref["fixed"])
    assert fr.shape == ref["free"].shape
    assert np.max(np.abs(fr - ref["free"]) / np.maximum(np.abs(ref["free"]).max(axis=1, keepdims=True), 1e-300)) < 1e-7
    assert abs(cost[0, 0] - ref["cost"]) <= 1e-9 * ref["cost"]


@pytest.mark.gpu
def test_cpp_api_on_gpu(tmp_path, gpu_ctx):
    exe = _gxx_build(tmp_path)
    r = subprocess.run([exe, "device"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
