#!/usr/bin/env python3
"""Register and instruction budget of each pass of the DL kernel, from the device assembly.

The DL kernel (csrc/mtg_solve_dl.inc) inlines up to four passes; the pattern pass must not pay for
the others (their spills belong in their cold branches).  This builds the kernel unit with only the
passes named kept (the other passes' calls cut out of a copy of the source in a temp directory, the
product source untouched) and prints VGPRs / AGPRs / scratch / the kernel's instruction count.

  python scripts/pass_isa.py [--unit n10_d3] [--r 4] [--src DIR] pattern ends general fallback all
"""
import argparse
import os
import re
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mav_trajectory_generation_cmake_amd", "csrc")
CALLS = {
    "pattern": r"dl_run_pass<DC, AL16>\(c, a, w, E, own, 0, lds, tph\);",
    "ends": r"dl_ends_pass<N, R, KMAX, D, AL16>\(eown\);",
    "general": r"dl_general_pass<N, R, KMAX, D, AL16>\(gown\);",
    "fallback": r"dl_fallback<N, R, D>\(a, w\.pair0, w\.nvt, __builtin_amdgcn_ballot_w64\(fown\), lds\);",
}


def build(keep, unit, r, src):
    tmp = tempfile.mkdtemp(prefix="pass_isa_")
    try:
        for f in os.listdir(src):
            if f.endswith((".inc", ".h", ".hip")):
                shutil.copy(os.path.join(src, f), tmp)
        p = os.path.join(tmp, "mtg_solve_dl.inc")
        s = open(p).read()
        for name, pat in CALLS.items():
            if name not in keep:
                s, n = re.subn(pat, "(void)0;", s)
                assert n == 1, (name, n)
        # a marker after the pattern pass: the instructions laid out before it are the pattern pass's
        mark = "  if (__builtin_expect(__builtin_amdgcn_ballot_w64(eown) != 0, 0)) {"
        assert s.count(mark) == 1
        s = s.replace(mark, '  asm volatile("; MTG_PATTERN_PASS_END" ::: "memory");\n' + mark)
        open(p, "w").write(s)
        out = os.path.join(tmp, "k.s")
        res = subprocess.run(["/opt/rocm/llvm/bin/clang++", "-I", os.path.join(ROOT, "include"), "-I", tmp, "-O3",
                              "-DNDEBUG", "-std=gnu++17", "--offload-arch=gfx950", "-fPIC", "--offload-device-only",
                              "-S", "-Rpass-analysis=kernel-resource-usage", "-o", out, "-x", "hip",
                              os.path.join(tmp, "mtg_solve_dl_%s.hip" % unit)], capture_output=True, text=True)
        if res.returncode:
            raise SystemExit(res.stderr[-3000:])
        asm = open(out).read()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    name = "solve_dl_kernelILi%sELi%dELi" % (unit.split("_")[0][1:], r)
    # the instantiation with the 16-B aligned output and plain stores (AL16 = 1; POL env: 2, sc1 stores)
    m = re.search(r"^(_ZN3mtg15%s\w*ELi%sEEEvNS_10DlKernArgsE):[^\n]*\n(.*?)^\.Lfunc_end"
                  % (name, os.environ.get("POL", "1")), asm, re.S | re.M)
    body = m.group(2)
    lines = body.splitlines()
    isins = [bool(re.match(r"^\s+[a-z_][a-z0-9_.]*\b", l)) and not l.strip().startswith(".") for l in lines]
    ins = [l for l, k in zip(lines, isins) if k]
    endm = [i for i, l in enumerate(lines) if "MTG_PATTERN_PASS_END" in l]
    head = [l for l, k in zip(lines[:endm[0]], isins) if k] if endm else []
    meta = {}
    rr = re.findall(r"remark:\s+Function Name: (\S+).*?VGPRs: (\d+).*?AGPRs: (\d+).*?ScratchSize \[bytes/lane\]: (\d+)",
                    res.stderr, re.S)
    for fn, v, a, sc in rr:
        if fn == m.group(1):
            meta = {"vgpr": int(v), "agpr": int(a), "scratch": int(sc)}
    nscr = sum(1 for l in ins if "scratch_" in l)
    return dict(meta, instructions=len(ins), scratch_ops=nscr, before_mark=len(head),
                scratch_ops_before_mark=sum(1 for l in head if "scratch_" in l),
                valu_f64=sum(1 for l in ins if re.match(r"^\s+v_\w*_f64", l)),
                stores=sum(1 for l in ins if "buffer_store" in l))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--unit", default="n10_d3")
    ap.add_argument("--r", type=int, default=4)
    ap.add_argument("--src", default=CSRC)
    ap.add_argument("sets", nargs="+")
    a = ap.parse_args()
    for s in a.sets:
        keep = set(CALLS) if s == "all" else set(s.split("+"))
        print(s, build(keep, a.unit, a.r, a.src))


if __name__ == "__main__":
    main()
