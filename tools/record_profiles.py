#!/usr/bin/env python3
"""Copy one GPU round's bench lines, rocprofv3 kernel statistics and PMC passes into
profiles/<round>/ and refresh profiles/pmc_traffic.json (the `traffic` figure bench.py reports).

  python tools/record_profiles.py <tag> <round-dir>        e.g.  r03g r03

Inputs (gpurun_out/, written by scripts/gpu_round.sh and scripts/gpu_pmc_round.sh):
  bench_<cfg>_<tag>.json, prof_<cfg>_<tag>/run_kernel_stats.csv,
  pmc_{fetch,write}_<cfg>_<tag>/run_counter_collection.csv, pmc_sq{a,b}_<cfg>_<tag>/...
Outputs: profiles/<round>/bench_<cfg>.json, <cfg>_kernel_stats.csv, pmc_summary.json,
summary.txt (bench kernel average vs the trace's, traffic / algorithmic, SQ ratios).
"""
import csv
import json
import os
import shutil
import statistics
import sys

CFGS = ("c1", "c1_s1536", "c2", "c2slot", "c2ethmix", "c2tx", "c2tx_nw", "c2nat", "c2v6", "c2eth", "c3_reasm", "c3_reasm6", "c3_reasm_il",
        "c3_reasm_retx", "c3_reasm_576", "c3", "c3_64k", "c3_frag", "c4")


PRODUCT = ("csum", "reassemble", "reasm_")        # the library's kernels


def product(name):
    return any(k in name for k in PRODUCT)


def step_kernels(counts):
    """The kernels of one step: the product kernels with the most dispatches (a step of the IPv4
    reassembly is two launches, the flat gather and its finish, dispatched equally often)."""
    top = max(counts.values())
    return sorted(k for k, v in counts.items() if v == top)


def counter_medians(path):
    """Per counter, the sum over the step's kernels of each kernel's median over its dispatches."""
    rows = [x for x in csv.DictReader(open(path)) if product(x["Kernel_Name"])]
    disp = {}
    for x in rows:
        disp.setdefault(x["Kernel_Name"], set()).add(x.get("Dispatch_Id", x.get("Correlation_Id")))
    kerns = step_kernels({k: len(v) for k, v in disp.items()})
    by = {}
    for x in rows:
        if x["Kernel_Name"] in kerns:
            by.setdefault((x["Kernel_Name"], x["Counter_Name"]), []).append(float(x["Counter_Value"]))
    med = {}
    for (k, c), v in by.items():
        med[c] = med.get(c, 0.0) + statistics.median(v)
    return " + ".join(kerns), med


def bench_line(path):
    """The bench JSON line printed in a log (the profiled process's own line)."""
    line = None
    if os.path.exists(path):
        for x in open(path, errors="replace"):
            x = x.strip()
            if x.startswith("{") and '"metric"' in x:
                line = json.loads(x)
    return line


def timed_trace(src, tcfg, tag, bench, dst):
    """Timed-region statistics of one rocprofv3 kernel trace (prof_<tcfg>_<tag>/): the last `steps`
    dispatches of the timed kernel, against the bench line printed by the SAME traced process (its
    HIP events ran under the profiler too) and against the unprofiled bench line of the round.
    Writes <tcfg>_timed.txt (JSON) and <tcfg>_kernel_stats.csv; returns the trace mean (us)."""
    d = os.path.join(src, f"prof_{tcfg}_{tag}")
    if not os.path.isdir(d):
        return None
    shutil.copy(os.path.join(d, "run_kernel_stats.csv"), os.path.join(dst, f"{tcfg}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))
    rows = [r for r in rows if product(r["Name"])]
    tr = os.path.join(d, "run_kernel_trace.csv")
    same = bench_line(os.path.join(src, f"prof_{tcfg}_{tag}.log"))
    ref = same or bench
    if not (rows and os.path.exists(tr) and ref):
        return None
    # the timed region: the last `steps` dispatches of the step's kernels (the stats file's average
    # also holds the setup and verification launches); a step of several kernels is their sum
    tops = step_kernels({r["Name"]: int(r["Calls"]) for r in rows})
    trace = [x for x in csv.DictReader(open(tr)) if x["Kernel_Name"] in tops]
    trace_us, firsts, ends, n_ts = 0.0, [], [], 0
    for k in tops:
        ts = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in trace if x["Kernel_Name"] == k)
        last = ts[-ref["steps"]:]
        trace_us += sum(e - b for b, e in last) / len(last) / 1e3
        firsts.append(last[0][0])
        ends.append(last[-1][1])
        n_ts = len(ts)
    bracket_us = (max(ends) - min(firsts)) / len(last) / 1e3
    algo = ref["roofline"]["algorithmic_bytes_per_launch"]
    peak = ref["roofline"]["peak"]
    top = " + ".join(tops)
    out = {"kernel": top, "timed_dispatches": len(last), "dispatches_total": n_ts,
           "trace_avg_us": round(trace_us, 3), "trace_bracket_us": round(bracket_us, 3),
           "frac_from_trace": round(algo / (trace_us * 1e3) / peak, 4),
           "frac_from_trace_bracket": round(algo / (bracket_us * 1e3) / peak, 4),
           "algorithmic_bytes_per_launch": algo}
    if same:
        out["same_process_line_kernel_avg_us"] = same["roofline"]["kernel_avg_us"]
        out["same_process_line_frac"] = same["roofline"]["frac"]
        out["same_process_launch"] = same["config"]["launch"]
    if bench:
        out["unprofiled_line_kernel_avg_us"] = bench["roofline"]["kernel_avg_us"]
        out["unprofiled_line_frac"] = bench["roofline"]["frac"]
    open(os.path.join(dst, f"{tcfg}_timed.txt"), "w").write(json.dumps(out, indent=1) + "\n")
    return trace_us


def main() -> None:
    tag, rnd = sys.argv[1], sys.argv[2]
    src = "gpurun_out"
    dst = os.path.join("profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    path = os.path.join("profiles", "pmc_traffic.json")
    rec = json.load(open(path)) if os.path.exists(path) else {}
    summary, pmc = [], {}
    for cfg in CFGS:
        bench = None
        f = os.path.join(src, f"bench_{cfg}_{tag}.json")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(dst, f"bench_{cfg}.json"))
            bench = json.loads(open(f).read().strip().splitlines()[-1])
        trace_us = None
        for tcfg in ((cfg, "c1ng") if cfg == "c1" else (cfg,)):
            t = timed_trace(src, tcfg, tag, bench, dst)
            if tcfg == cfg:
                trace_us = t
        r = {}
        for kind, c in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
            f = os.path.join(src, f"pmc_{kind}_{cfg}_{tag}", "run_counter_collection.csv")
            if os.path.exists(f):
                kern, med = counter_medians(f)
                r[c + "_kB_median"] = med[c]
                r["kernel"] = kern
        if "FETCH_SIZE_kB_median" in r and "WRITE_SIZE_kB_median" in r:
            r["hbm_read_bytes_per_launch"] = int(r["FETCH_SIZE_kB_median"] * 1024 * 2)
            r["hbm_write_bytes_per_launch"] = int(r["WRITE_SIZE_kB_median"] * 1024)
            r["hbm_bytes_per_launch"] = r["hbm_read_bytes_per_launch"] + r["hbm_write_bytes_per_launch"]
            if bench:
                algo = bench["roofline"]["algorithmic_bytes_per_launch"]
                r["algorithmic_bytes_per_launch"] = algo
                r["traffic_over_algorithmic"] = round(r["hbm_bytes_per_launch"] / algo, 3)
            r["round"] = rnd
            rec[cfg] = r
        sq = {}
        for p in ("sqa", "sqb"):
            f = os.path.join(src, f"pmc_{p}_{cfg}_{tag}", "run_counter_collection.csv")
            if os.path.exists(f):
                sq.update(counter_medians(f)[1])
        if sq:
            waves = sq.get("SQ_WAVES", 0) or 1
            wc = sq.get("SQ_WAVE_CYCLES", 0) or 1
            sq["VALU_insts_per_wave"] = round(sq.get("SQ_INSTS_VALU", 0) / waves, 1)
            sq["wait_any_frac"] = round(sq.get("SQ_WAIT_ANY", 0) / wc, 3)
            sq["wait_inst_any_frac"] = round(sq.get("SQ_WAIT_INST_ANY", 0) / wc, 3)
            sq["active_inst_any_frac"] = round(sq.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)
            pmc[cfg] = sq
        if bench:
            line = (f"{cfg:10s} value {bench['value']:9.2f} {bench['unit']}  kernel {bench['roofline']['kernel_avg_us']:8.2f} us"
                    f" (trace {trace_us:8.2f} us)" if trace_us else
                    f"{cfg:10s} value {bench['value']:9.2f} {bench['unit']}  kernel {bench['roofline']['kernel_avg_us']:8.2f} us")
            line += f"  frac {bench['roofline']['frac']:.4f}"
            if cfg in rec and rec[cfg].get("round") == rnd:
                line += (f"  traffic/algorithmic {rec[cfg]['traffic_over_algorithmic']}"
                         f"  write {rec[cfg]['hbm_write_bytes_per_launch'] / 1e6:.2f} MB")
            if bench.get("verified"):
                line += f"  verified {bench['verified']['frames']} frames, {bench['verified']['mismatches']} mismatches"
            summary.append(line)
    rec["_method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                      "`bench.py --config <c> --steps 20 --warmup 2`; median over the timed kernel's dispatches; "
                      "FETCH_SIZE (kB) x1024 x2 (calibrated to 128 B per 128-B line touched, tools/fetch_calib.py), "
                      "WRITE_SIZE (kB) x1024")
    json.dump(rec, open(path, "w"), indent=1)
    if pmc:
        json.dump(pmc, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
        for cfg, sq in pmc.items():
            summary.append(f"{cfg:10s} SQ: VALU insts/wave {sq['VALU_insts_per_wave']}, wait_any {sq['wait_any_frac']}, "
                           f"wait_inst_any {sq['wait_inst_any_frac']}, active_inst_any {sq['active_inst_any_frac']}, "
                           f"waves {int(sq.get('SQ_WAVES', 0))}")
    open(os.path.join(dst, "summary.txt"), "w").write("\n".join(summary) + "\n")
    print("\n".join(summary))


if __name__ == "__main__":
    main()
