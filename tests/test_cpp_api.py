"""The C++ drop-in header (include/mtg/trajectory_generation.hpp): compiles on CPU, runs on the GPU."""
import os
import shutil
import subprocess

import pytest

from mav_trajectory_generation_cmake_amd import _native as nat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_cpp_api.cpp")


def _build(tmp_path):
    cxx = shutil.which("g++") or "g++"
    exe = tmp_path / "test_cpp_api"
    libdir = os.path.dirname(nat.LIB_PATH)
    subprocess.run([cxx, "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    SRC, "-o", str(exe), "-L", libdir, "-lmtg", "-Wl,-rpath," + libdir], check=True)
    return exe


def test_cpp_header_compiles(tmp_path):
    assert _build(tmp_path).exists()


@pytest.mark.gpu
def test_cpp_api_on_gpu(tmp_path, gpu_ctx):
    exe = _build(tmp_path)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
