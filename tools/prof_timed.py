#!/usr/bin/env python3
"""Timed-region kernel statistics from a rocprofv3 kernel trace, so that a bench line's
`roofline.frac` can be re-derived from the profile of the same process.

  python tools/prof_timed.py <run_kernel_trace.csv> <bench line .json> [--out summary.json]

The bench's timed region is its last `steps` launches of the checksum kernel (warm-up
and untimed setup come first; the bench line names `steps`).  For those dispatches:
average / median / min / max duration, and the bracket (last end - first start) / steps,
which is what the HIP events in bench.py measure.  `frac_from_trace` = the bench line's
algorithmic bytes per launch / trace average / 8 TB/s.  The rocprofv3 --stats summary
(run_kernel_stats.csv) averages every dispatch of a kernel name, setup and warm-up
included; this separates the timed ones.
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--out")
    a = ap.parse_args()
    line = None
    with open(a.bench) as f:
        for x in f:
            x = x.strip()
            if x.startswith("{") and '"metric"' in x:
                line = json.loads(x)
    if line is None:
        raise SystemExit(f"no bench line in {a.bench}")
    steps = int(line["steps"])
    rows = list(csv.DictReader(open(a.trace)))
    by = {}
    for r in rows:
        nm = r["Kernel_Name"]
        if "csum" in nm or "forward_kernel" in nm or "reassemble" in nm:
            by.setdefault(nm, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    kern = max(by, key=lambda k: len(by[k]))
    disp = sorted(by[kern])
    timed = disp[-steps:]
    durs = [e - s for s, e in timed]
    avg = statistics.fmean(durs)
    bracket = (timed[-1][1] - timed[0][0]) / len(timed)
    algo = line["roofline"]["algorithmic_bytes_per_launch"]
    peak = line["roofline"]["peak"]
    out = {
        "kernel": kern, "dispatches_total": len(disp), "timed_dispatches": len(timed),
        "avg_ns": round(avg, 1), "median_ns": statistics.median(durs), "min_ns": min(durs), "max_ns": max(durs),
        "bracket_ns_per_launch": round(bracket, 1),
        "all_dispatches_avg_ns": round(statistics.fmean(e - s for s, e in disp), 1),
        "bench_kernel_avg_us": line["roofline"].get("kernel_avg_us"),
        "bench_frac": line["roofline"]["frac"],
        "frac_from_trace": round(algo / (avg * 1e-9) / 1e9 / peak, 4),
        "frac_from_trace_bracket": round(algo / (bracket * 1e-9) / 1e9 / peak, 4),
        "algorithmic_bytes_per_launch": algo,
    }
    js = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
