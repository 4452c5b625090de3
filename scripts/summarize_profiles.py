#!/usr/bin/env python3
"""Summarise rocprofv3 output (scripts/profile.sh -> gpurun_out/prof_b<B>/) into profiles/.

For each batch size B:
  profiles/<tag>_b<B>_kernel_stats.csv   copy of rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_b<B>_pmc.json           per-kernel PMC means (separate passes per counter group)
and merges profiles/pmc_traffic.json {kernel: {B: {"hbm_bytes_per_launch", ...}}}, which
bench.py reports as roofline.traffic.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (both reported in KiB): the doubling is the
gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md "HBM [CDNA4]" (FETCH_SIZE = TCC_EA0_RDREQ x 64 B
with 128-B requests).  Infinity-Cache (L3) hits are counted by these counters, so at sizes whose
inputs stay L3-resident between launches this over-states true HBM bytes.

usage: summarize_profiles.py TAG B [B ...]      (reads gpurun_out/prof<SRC>_b<B>, SRC from $PROF_SRC;
       $WORKLOAD names the bench workload profiled, default config2, and $PATTERN its vertex pattern
       (bench.py --pattern), default generator: traffic is keyed "<kernel>|<workload>|<pattern>" and
       stamped with the kernel sources' digest (bench.csrc_digest), so a capture is not quoted for
       another workload, pattern or build)
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def counter_means(path, skip_first=2):
    """Mean of each counter per kernel over dispatches, skipping the first `skip_first` dispatches
    of each kernel (warm-up)."""
    per = {}
    seen = {}
    rows = _rows(path)
    # only the bench's own launches: per kernel, the dispatches with the largest grid (the
    # end_to_end leg's pipeline chunks launch the same kernel on smaller grids)
    grid = {}
    for r in rows:
        grid[r["Kernel_Name"]] = max(grid.get(r["Kernel_Name"], 0), int(r.get("Grid_Size", 0) or 0))
    rows = [r for r in rows if int(r.get("Grid_Size", 0) or 0) == grid[r["Kernel_Name"]]]
    for r in rows:
        k = r["Kernel_Name"]
        if k.startswith("__amd_rocclr"):
            continue  # runtime copies
        key = (k, r["Counter_Name"])
        seen[key] = seen.get(key, 0) + 1
        if seen[key] <= skip_first:
            continue
        per.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in per.items()}
    for k in out:
        out[k]["grid"] = grid[k]
    return out


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "").replace("mtg::", "").split("<")[0]


def main():
    sys.path.insert(0, ROOT)
    import bench
    digest = bench.csrc_digest()
    tag = sys.argv[1]
    batches = sys.argv[2:]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    tpath = os.path.join(prof, "pmc_traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    for B in batches:
        src = os.path.join(ROOT, "gpurun_out", "prof%s_b%s" % (os.environ.get("PROF_SRC", ""), B))
        stats = os.path.join(src, "trace", "run_kernel_stats.csv")
        shutil.copy(stats, os.path.join(prof, "%s_b%s_kernel_stats.csv" % (tag, B)))
        pmc = {}
        for group in ("pmc_fetch", "pmc_write", "pmc_l2"):
            p = os.path.join(src, group, "run_counter_collection.csv")
            if os.path.exists(p):
                for k, d in counter_means(p).items():
                    pmc.setdefault(k, {}).update(d)
        summary = {"batch": int(B), "source": "rocprofv3 --kernel-trace --pmc, one pass per counter group "
                                              "(scripts/profile.sh)", "kernels": {}}
        # per short kernel name, the instantiation with the largest grid is the bench's own launch
        # (the end_to_end leg's chunks can run another instantiation of the same kernel)
        best = {}
        for k, d in pmc.items():
            sk = short(k)
            if sk not in best or d.get("grid", 0) > pmc[best[sk]].get("grid", 0):
                best[sk] = k
        for k, d in pmc.items():
            ent = dict(d)
            if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
                ent["hbm_bytes_per_launch"] = 2.0 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
            if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
                ent["l2_hit_rate"] = d["TCC_HIT_sum"] / max(d["TCC_HIT_sum"] + d["TCC_MISS_sum"], 1.0)
            summary["kernels"][k] = ent
            if "hbm_bytes_per_launch" in ent and best.get(short(k)) == k:
                key = bench.traffic_key(short(k), os.environ.get("WORKLOAD", "config2"),
                                        os.environ.get("PATTERN", "generator"))
                traffic.setdefault(key, {})[str(B)] = {
                    "csrc_sha256": digest,
                    "hbm_bytes_per_launch": ent["hbm_bytes_per_launch"],
                    "fetch_kib_raw": d["FETCH_SIZE"], "write_kib": d["WRITE_SIZE"],
                    "l2_hit_rate": ent.get("l2_hit_rate"), "profile": "%s_b%s_pmc.json" % (tag, B)}
        with open(os.path.join(prof, "%s_b%s_pmc.json" % (tag, B)), "w") as f:
            json.dump(summary, f, indent=1)
        for row in _rows(stats):
            print(B, row["Name"][:60], "calls", row["Calls"], "avg_us %.2f" % (float(row["AverageNs"]) / 1e3))
        for k, e in summary["kernels"].items():
            print(B, k[:60], {a: (round(b, 3) if isinstance(b, float) else b) for a, b in e.items()})
    with open(tpath, "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
