"""Average PMC counters per kernel (one row per kernel name and grid size) from
rocprofv3 csv passes, with the derived occupancy / issue split:
  waves          = SQ_WAVES
  gpu_cycles     = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs, MI355X_MICROARCH.md "DVFS")
  busy_us        = gpu_cycles / 2.4 GHz (the dispatch's active span, profiler overhead included)
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x gpu_cycles)
  waves_per_simd = 4 x SQ_WAVE_CYCLES / (1024 SIMDs x gpu_cycles)  (SQ_WAVE_CYCLES counts quad-cycles)
  wait / issue-stall / active = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
usage: python tools/pmc_summary.py <dir with p*/ passes>
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = (row["Kernel_Name"][:70], row.get("Grid_Size", ""))
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        meta[k] = {x: row.get(x) for x in ("Workgroup_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
                                           "LDS_Block_Size") if row.get(x) is not None}
for k, cs in acc.items():
    print(f"{k[0]}  grid {k[1]}  {meta.get(k, {})}")
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    for c, v in sorted(cs.items()):
        # each dispatch reports one value per counter (summed over dims by rocprofv3)
        print(f"   {c:28s} {avg[c]:16.1f}  (n={len(v)})")
    g = avg.get("GRBM_GUI_ACTIVE")
    g = g / 8.0 if g else g
    wc = avg.get("SQ_WAVE_CYCLES")
    if g:
        der = {"busy_us": g / 2400.0}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
            der["mfma_busy"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * g)
        if wc:
            der["waves_per_simd"] = 4.0 * wc / (1024.0 * g)
            for c, n in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "issue_stall"),
                         ("SQ_ACTIVE_INST_ANY", "active")):
                if c in avg:
                    der[n] = avg[c] / wc
        print("   derived " + "  ".join(f"{n} {v:.3f}" for n, v in der.items()))
