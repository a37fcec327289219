#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (one directory per run under ROOT): per counter, the median over
the checksum kernel's dispatches (the kernel with the most dispatches in the run)."""
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
res = {}
for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
    name = os.path.basename(os.path.dirname(f))
    rows = [r for r in csv.DictReader(open(f)) if "csum" in r["Kernel_Name"] or "reassemble" in r["Kernel_Name"]]
    # the measured kernel: the one with the most dispatches (setup launches differ)
    counts = {}
    for r in rows:
        counts[r["Kernel_Name"]] = counts.get(r["Kernel_Name"], 0) + 1
    if counts:
        top = max(counts, key=counts.get)
        rows = [r for r in rows if r["Kernel_Name"] == top]
    per = {}
    for r in rows:
        per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    d = res.setdefault(name, {})
    for k, v in per.items():
        d[k] = statistics.median(v)
    if rows:
        d["_kernel"] = rows[0]["Kernel_Name"][:70]
        d["_vgpr"] = rows[0]["VGPR_Count"]
        d["_lds"] = rows[0]["LDS_Block_Size"]
for name, d in res.items():
    print(f"== {name}  {d.get('_kernel')}  vgpr={d.get('_vgpr')} lds={d.get('_lds')}")
    for k in sorted(d):
        if not k.startswith("_"):
            print(f"   {k:34s} {d[k]:16.1f}")
    wc = d.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM"):
            if k in d:
                print(f"   {k + ' / WAVE_CYCLES':34s} {d[k] / wc:16.3f}")
    if "SQ_LEVEL_WAVES" in d and "SQ_BUSY_CYCLES" in d:
        print(f"   {'avg waves (LEVEL/BUSY)':34s} {d['SQ_LEVEL_WAVES'] / d['SQ_BUSY_CYCLES']:16.2f}")
