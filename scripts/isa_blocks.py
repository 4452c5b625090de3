#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in a device assembly file (hipcc -S
--cuda-device-only): all / VALU / SALU / LDS / global-memory instructions and the branches that end
each block, so that a loop body's cost can be read off without a GPU.

  python scripts/isa_blocks.py dl3.s 'solve_dl_kernelILi10ELi4ELi10ELi3E' [--min 20]
"""
import argparse
import re


def kernel_body(lines, key):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", l) and key in l.split(":")[0]:
            start = i
        elif start is not None and l.strip().startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit("kernel %r not found" % key)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--min", type=int, default=0, help="only blocks with at least this many instructions")
    args = ap.parse_args()
    body = kernel_body(open(args.asm).read().split("\n"), args.kernel)
    blocks = []
    cur = None
    for l in body:
        m = re.match(r"^(\.LBB\S+):", l) or re.match(r"^; (%bb\.\d+):", l)
        if m or cur is None:
            cur = {"name": m.group(1) if m else "entry", "all": 0, "v": 0, "f64": 0, "s": 0, "ds": 0, "glb": 0,
                   "br": []}
            blocks.append(cur)
            if m:
                continue
        t = l.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        cur["all"] += 1
        if op.startswith("v_"):
            cur["v"] += 1
            if "_f64" in op:
                cur["f64"] += 1
        elif op.startswith("s_"):
            cur["s"] += 1
            if op.startswith("s_cbranch") or op == "s_branch":
                cur["br"].append(t)
        elif op.startswith("ds_"):
            cur["ds"] += 1
        elif op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
            cur["glb"] += 1
    tot = {k: sum(b[k] for b in blocks) for k in ("all", "v", "f64", "s", "ds", "glb")}
    print("%-14s %6s %6s %6s %6s %5s %5s  branches" % ("block", "all", "valu", "f64", "salu", "lds", "glob"))
    for b in blocks:
        if b["all"] >= args.min:
            print("%-14s %6d %6d %6d %6d %5d %5d  %s" % (b["name"], b["all"], b["v"], b["f64"], b["s"], b["ds"], b["glb"],
                                                    " | ".join(b["br"])))
    print("%-14s %6d %6d %6d %6d %5d %5d" % ("total", tot["all"], tot["v"], tot["f64"], tot["s"], tot["ds"], tot["glb"]))


if __name__ == "__main__":
    main()
