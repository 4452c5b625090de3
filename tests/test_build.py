"""CPU checks on the gfx950 code the HIP sources compile to (hipcc cross-compiles without a GPU)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mav_trajectory_generation_cmake_amd", "csrc")

hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
pytestmark = pytest.mark.skipif(not os.path.exists(hipcc), reason="hipcc not available")


def _device_asm(src, tmp_path):
    out = tmp_path / (os.path.basename(src) + ".s")
    inc = os.path.join(os.path.dirname(os.path.dirname(CSRC)), "include")
    subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-I", inc,
                    "-I", CSRC, os.path.join(CSRC, src), "-o", str(out)], check=True, capture_output=True)
    return out.read_text()


def _kernel_bodies(asm, prefix):
    bodies = {}
    for m in re.finditer(r"^(%s\w*):" % prefix, asm, flags=re.M):
        end = asm.find("s_endpgm", m.end())
        bodies[m.group(1)] = asm[m.end():end]
    return bodies


def test_evaluate_range_has_no_fma(tmp_path):
    """Polynomial::evaluate (polynomial.h:138-151) multiplies then adds; an FMA would change the
    last bit and break bit-exact parity of evaluateRange with the reference."""
    asm = _device_asm("mtg_eval.hip", tmp_path)
    bodies = _kernel_bodies(asm, r"_ZN3mtg17eval_range_kernel")
    # N = 2, 4, ..., 12 x derivative 0..4 and the runtime-derivative variant x (D = 3, D = 3 stored-run
    # only (ST), run-time D)
    assert len(bodies) == 108
    # the producer / consumer form of the stored-run D = 3 kernel: N x derivative
    pc = _kernel_bodies(asm, r"_ZN3mtg20eval_range_pc_kernel")
    assert len(pc) == 36
    bodies.update(pc)
    for name, body in bodies.items():
        # f64 FMAs are allowed only as the compiler's f64 -> int64 conversion idiom (x - 2^32 hi,
        # constant 0xc1f00000) in the clock's integer run arithmetic; f32 FMAs belong to its
        # integer-division emulation.  Any other f64 FMA would be a contracted Horner step.
        bad = [ln for ln in body.splitlines() if re.search(r"v_fmac?_f64", ln) and "0xc1f00000" not in ln]
        assert not bad, (name, bad[:3])
