#!/usr/bin/env python3
"""Copy one GPU round's rocprofv3 summaries + bench lines into profiles/<round>/ and
refresh profiles/pmc_traffic.json (the `traffic` figure bench.py reports).

  python tools/record_profiles.py <tag> <round-dir>      e.g.  r01c r01
"""
import csv
import json
import os
import shutil
import statistics
import sys

tag, rnd = sys.argv[1], sys.argv[2]
src = "gpurun_out"
dst = os.path.join("profiles", rnd)
os.makedirs(dst, exist_ok=True)
for cfg in ("c1", "c2", "c2v6"):
    d = os.path.join(src, f"prof_{cfg}_{tag}")
    if os.path.isdir(d):
        shutil.copy(os.path.join(d, "run_kernel_stats.csv"), os.path.join(dst, f"{cfg}_kernel_stats.csv"))
for cfg in ("c1", "c2", "c2tx", "c2v6", "c3", "c3_64k", "c3_frag"):
    f = os.path.join(src, f"bench_{cfg}_{tag}.json")
    if os.path.exists(f):
        shutil.copy(f, os.path.join(dst, f"bench_{cfg}.json"))
path = os.path.join("profiles", "pmc_traffic.json")
rec = json.load(open(path)) if os.path.exists(path) else {}
for cfg in ("c1", "c2", "c2v6"):
    r = {}
    for kind, c in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        f = os.path.join(src, f"pmc_{kind}_{cfg}_{tag}", "run_counter_collection.csv")
        if not os.path.exists(f):
            break
        rows = list(csv.DictReader(open(f)))
        # the timed kernel = the checksum kernel with the most dispatches
        names = {}
        for x in rows:
            if "csum" in x["Kernel_Name"]:
                names[x["Kernel_Name"]] = names.get(x["Kernel_Name"], 0) + 1
        kern = max(names, key=names.get)
        r[c + "_kB_median"] = statistics.median(float(x["Counter_Value"]) for x in rows if x["Kernel_Name"] == kern)
        r["kernel"] = kern
    else:
        r["hbm_read_bytes_per_launch"] = int(r["FETCH_SIZE_kB_median"] * 1024 * 2)
        r["hbm_write_bytes_per_launch"] = int(r["WRITE_SIZE_kB_median"] * 1024)
        r["hbm_bytes_per_launch"] = r["hbm_read_bytes_per_launch"] + r["hbm_write_bytes_per_launch"]
        r["round"] = rnd
        rec[cfg] = r
rec["_method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                  "`bench.py --config <c> --steps 20`; median over the timed checksum kernel's dispatches; "
                  "FETCH_SIZE (kB) x1024 x2 (gfx950 reports half of wide coalesced reads, MI355X_MICROARCH.md "
                  "HBM section), WRITE_SIZE (kB) x1024")
json.dump(rec, open(path, "w"), indent=1)
print(json.dumps({k: v for k, v in rec.items() if k != "_method"}, indent=1))
