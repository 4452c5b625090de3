#!/usr/bin/env python3
"""Print per-dispatch means of the PMC counters collected by scripts/pmc_sq.sh for one kernel."""
import collections
import csv
import glob
import sys

d = collections.defaultdict(list)
meta = {}
rows = []
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    rows += [r for r in csv.DictReader(open(f)) if sys.argv[2] in r["Kernel_Name"]]
# only the bench's own launches (the largest grid): the bench's end-to-end leg runs the same kernel on
# smaller pipelined chunks, which must not be averaged in
gmax = max(int(r["Grid_Size"]) for r in rows)
for r in rows:
    if int(r["Grid_Size"]) == gmax:
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta = {k: r[k] for k in ("LDS_Block_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Grid_Size")}
m = {k: sum(v[2:]) / max(len(v[2:]), 1) for k, v in d.items()}
for k in sorted(m):
    print("%-24s %.4g" % (k, m[k]))
print(meta)
w = m.get("SQ_WAVES", 0)
if w:
    print("per wave: VALU %.0f  SALU %.0f  LDS %.0f  SMEM %.0f" % tuple(m.get(k, 0) / w for k in
          ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM")))
if "SQ_WAVE_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
    simd_cycles = m["GRBM_GUI_ACTIVE"] / 8 * 256 * 4
    print("resident waves/SIMD %.2f   VALU busy %.2f" % (m["SQ_WAVE_CYCLES"] * 4 / simd_cycles,
                                                       m.get("SQ_ACTIVE_INST_VALU", 0) * 4 / simd_cycles))
    tot = m["SQ_WAVE_CYCLES"]
    print("wave time: active %.2f  wait_any %.2f  wait_inst %.2f" % (m["SQ_ACTIVE_INST_ANY"] / tot,
                                                                    m["SQ_WAIT_ANY"] / tot,
                                                                    m["SQ_WAIT_INST_ANY"] / tot))
