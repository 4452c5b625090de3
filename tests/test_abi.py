"""CPU tests of the drop-in boundary (include/mtg.h <-> libmav_trajectory_generation.so <-> _native.py).

No compute calls here: these run without a GPU and check that the C ABI library
loads, exports exactly what the header declares, validates arguments and
reports "no device" loudly (there is no CPU fallback in the product path)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from mav_trajectory_generation_cmake_amd import _native as nat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(nat.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(mtg_[a-z0-9_]+)\s*\(", src))


def _header_defines():
    out = {}
    for m in re.finditer(r"#define\s+(MTG_[A-Z0-9_]+)\s+\(?(-?\d+)u?\)?", open(nat.HEADER).read()):
        out[m.group(1)] = int(m.group(2))
    return out


def test_header_and_binding_agree():
    assert _header_functions() == set(nat.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = nat.load()
    for name in _header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", nat.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln and ln.split()[-1].startswith("mtg_")}
    assert exported == _header_functions()


def test_constants_match_header():
    for name, val in _header_defines().items():
        if name in ("MTG_H_",):
            continue
        if hasattr(nat, name):
            assert getattr(nat, name) == val, name
    assert nat.load().mtg_abi_version() == _header_defines()["MTG_ABI_VERSION"]


def test_status_strings():
    for code in (0, -1, -2, -3, -4, -5, -6, -7, -8):
        assert nat.status_string(code)
    assert nat.status_string(-99)


def test_one_hip_runtime_in_process():
    """The library must bind to the same libamdhip64 as torch (see _native._share_torch_runtime)."""
    pytest.importorskip("torch")
    nat.load()
    assert len(nat.hip_runtimes_mapped()) == 1, nat.hip_runtimes_mapped()


def test_null_context_rejected():
    lib = nat.load()
    z = np.zeros(64)
    m = np.zeros(64, np.uint8)
    a = z.ctypes.data
    assert lib.mtg_solve_linear_batch(None, 10, 3, 1, 4, 1, a, m.ctypes.data, a, a, None, None, None, None,
                                      0) == nat.MTG_ERR_INVALID_ARGUMENT
    assert lib.mtg_time_sweep_batch(None, 10, 3, 1, 4, 1, a, m.ctypes.data, a, 1, a, a, None,
                                    0) == nat.MTG_ERR_INVALID_ARGUMENT
    assert lib.mtg_set_stream(None, None) == nat.MTG_ERR_INVALID_ARGUMENT
    assert lib.mtg_synchronize(None) == nat.MTG_ERR_INVALID_ARGUMENT
    assert lib.mtg_enable_timing(None, 4) == nat.MTG_ERR_INVALID_ARGUMENT
    assert lib.mtg_destroy(None) == nat.MTG_OK
    assert lib.mtg_create(0, None) == nat.MTG_ERR_INVALID_ARGUMENT
    assert lib.mtg_device_count(None) == nat.MTG_ERR_INVALID_ARGUMENT


@pytest.mark.skipif(nat.device_count() > 0, reason="checks the no-device path")
def test_no_device_fails_loudly():
    from mav_trajectory_generation_cmake_amd import Context
    with pytest.raises(nat.MTGError) as e:
        Context(0)
    assert e.value.code == nat.MTG_ERR_NO_DEVICE


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(nat.MTGError):
        nat.load(str(tmp_path / "libmav_trajectory_generation.so"))


def test_host_generator_argument_errors():
    lib = nat.load()
    v = np.zeros(1000)
    m = np.zeros(100, np.uint8)
    t = np.zeros(100)
    assert lib.mtg_host_random_vertices_path_batch(10, 3, 0, 5.0, 4, 0, 1, 2.0, 2.0, 6.5, v.ctypes.data,
                                                   m.ctypes.data, t.ctypes.data, 1) != nat.MTG_OK
    assert lib.mtg_host_random_vertices_path_batch(11, 3, 2, 5.0, 4, 0, 1, 2.0, 2.0, 6.5, v.ctypes.data,
                                                   m.ctypes.data, t.ctypes.data, 1) != nat.MTG_OK


def test_cpp_header_compiles_with_c_compiler(tmp_path):
    """include/mtg.h is plain C: a C99 translation unit that includes it compiles and links."""
    c = tmp_path / "t.c"
    c.write_text('#include "mtg.h"\nint main(void){ return mtg_abi_version() == MTG_ABI_VERSION ? 0 : 1; }\n')
    exe = tmp_path / "t"
    libdir = os.path.dirname(nat.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c), "-o",
                    str(exe), "-L", libdir, "-lmav_trajectory_generation", "-Wl,-rpath," + libdir], check=True)
    assert subprocess.run([str(exe)]).returncode == 0


def test_solve_kernel_selection():
    """mtg_solve_kernel (host-only query): the register column kernel by default for K <= 12 (N = 12:
    K <= 20), the dimension-lane kernel with MTG_FLAG_DL_KERNEL where it applies, the long-chain
    dimension-lane kernel or the general kernel beyond, errors for rejected shapes; the retired lane / IP flag bits (16, 32) are ignored."""
    from mav_trajectory_generation_cmake_amd import _native as nat
    lib = nat.load()
    dl, col, gen, split = (nat.MTG_KERNEL_DL, nat.MTG_KERNEL_COLUMN, nat.MTG_KERNEL_GENERAL,
                           nat.MTG_KERNEL_SPLIT)
    L = nat.MTG_FLAG_DL_KERNEL
    assert lib.mtg_solve_kernel(10, 3, 10, 4, nat.MTG_FLAG_COLUMN_KERNEL) == col  # config 2 / 3, column A/B
    assert lib.mtg_solve_kernel(12, 3, 20, 3, 0) == nat.MTG_KERNEL_DL  # config 4 (round 4)
    assert lib.mtg_solve_kernel(12, 3, 20, 3, nat.MTG_FLAG_COLUMN_KERNEL) == col
    assert lib.mtg_solve_kernel(12, 3, 18, 3, 0) == col  # the DL kernel is built for K = 20 at N = 12
    assert lib.mtg_solve_kernel(4, 3, 10, 1, 0) == col
    assert lib.mtg_solve_kernel(10, 3, 10, 4, L) == dl
    assert lib.mtg_solve_kernel(10, 1, 10, 1, L) == dl
    assert lib.mtg_solve_kernel(10, 4, 10, 3, L) == dl
    assert lib.mtg_solve_kernel(10, 3, 1, 4, L) == col    # K != 10: no DL kernel
    assert lib.mtg_solve_kernel(8, 1, 12, 3, L) == col
    assert lib.mtg_solve_kernel(10, 5, 10, 4, L) == col   # D > 4: no DL kernel
    assert lib.mtg_solve_kernel(10, 3, 10, 0, L) == col   # r = 0: no translation trick
    for retired in (16, 32):
        assert lib.mtg_solve_kernel(10, 3, 10, 4, retired) == nat.MTG_KERNEL_DL
    assert lib.mtg_solve_kernel(12, 3, 20, 3, L) == dl
    assert lib.mtg_solve_kernel(12, 5, 20, 3, L) == col  # D > 4
    # K outside both the DL kernel's (10 / 20) and the column kernel's (N = 10: <= 10) ranges: the
    # long-chain DL kernel (round 6) where it applies (N = 10 / 12, D <= 4, r >= 1), else the general one
    dlx = nat.MTG_KERNEL_DLX
    assert lib.mtg_solve_kernel(10, 3, 12, 4, 0) == dlx
    assert lib.mtg_solve_kernel(10, 3, 11, 4, 0) == dlx
    assert lib.mtg_solve_kernel(10, 3, 100, 4, 0) == dlx  # the reference benchmark's K = 100
    assert lib.mtg_solve_kernel(10, 1, 101, 1, 0) == dlx
    assert lib.mtg_solve_kernel(12, 4, 21, 3, 0) == dlx
    assert lib.mtg_solve_kernel(10, 3, 50, 4, L) == dlx
    assert lib.mtg_solve_kernel(10, 3, 50, 4, nat.MTG_FLAG_COLUMN_KERNEL) == gen  # (no column kernel there)
    assert lib.mtg_solve_kernel(10, 3, 50, 4, nat.MTG_FLAG_GENERAL_KERNEL) == gen
    assert lib.mtg_solve_kernel(10, 3, 50, 0, 0) == gen   # r = 0
    assert lib.mtg_solve_kernel(10, 5, 50, 4, 0) == gen   # D > 4
    assert lib.mtg_solve_kernel(8, 3, 50, 3, 0) == dlx    # N = 8 / 6 beyond the column kernel's K <= 12
    assert lib.mtg_solve_kernel(6, 2, 13, 2, 0) == dlx
    assert lib.mtg_solve_kernel(8, 3, 12, 3, 0) == col
    assert lib.mtg_solve_kernel(4, 3, 50, 1, 0) == gen    # N = 4: the general kernel
    assert nat.solve_kernel(10, 3, 50, 4) == "solve_dlx_kernel"
    assert lib.mtg_solve_kernel(10, 3, 10, 4, nat.MTG_FLAG_GENERAL_KERNEL) == gen
    assert lib.mtg_solve_kernel(10, 3, 10, 4, nat.MTG_FLAG_SPLIT_KERNELS) == split
    assert lib.mtg_solve_kernel(10, 3, 13, 4, 0) == dlx
    # the dimension-lane kernel by default wherever it applies (N = 10, K = 10, D <= 4, r >= 1), at
    # every batch size (a trajectory's bits do not depend on the size of its call); the column flag
    # keeps the column kernel
    dl = nat.MTG_KERNEL_DL
    assert lib.mtg_solve_kernel(10, 3, 10, 4, 0) == dl
    for B in (1, 10, 1024, 2047, 2048, 8192, 10000):
        assert lib.mtg_solve_kernel_batch(10, 3, 10, 4, B, 0) == dl
    assert lib.mtg_solve_kernel_batch(10, 3, 10, 4, 125000, nat.MTG_FLAG_COLUMN_KERNEL) == col
    assert lib.mtg_solve_kernel_batch(10, 3, 10, 4, 10, nat.MTG_FLAG_DL_KERNEL) == dl
    assert lib.mtg_solve_kernel_batch(10, 3, 10, 0, 125000, 0) == col  # r = 0: no translation trick
    assert lib.mtg_solve_kernel_batch(10, 3, 8, 4, 125000, 0) == col   # K != 10
    assert lib.mtg_solve_kernel_batch(12, 3, 20, 3, 125000, 0) == dl
    assert lib.mtg_solve_kernel_batch(10, 3, 10, 4, 125000, nat.MTG_FLAG_SPLIT_KERNELS) == split
    assert nat.solve_kernel(10, 3, 10, 4, B=125000) == "solve_dl_kernel"
    assert lib.mtg_solve_kernel(10, 3, 50, 4, 0) == nat.MTG_KERNEL_DLX
    assert lib.mtg_solve_kernel(11, 3, 10, 4, 0) == nat.MTG_ERR_UNSUPPORTED_N
    assert lib.mtg_solve_kernel(10, 3, 10, 5, 0) == nat.MTG_ERR_BAD_DERIVATIVE
    assert nat.solve_kernel(10, 3, 10, 4) == "solve_dl_kernel"
    assert nat.solve_kernel(10, 3, 10, 4, L) == "solve_dl_kernel"
