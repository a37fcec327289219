#!/usr/bin/env python3
"""Thread sweep of the CPU baseline: the reference's own pico_checksum (oracle/_ref, built from
stack/pico_frame.c -O3 and -Os) over C1-shaped frames (1500 B, contiguous, DRAM-resident) on
1, 2, 4, 8 and 16 pthreads -- the host share a GPU box grants one GPU's job (OMP_NUM_THREADS=16;
the machine's other cores belong to other jobs, so the sweep stops there).

    python tools/cpu_sweep.py [--mib 375] [--seconds 3] [--out gpurun_out/cpu_sweep.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

GIB = 1 << 30


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=375)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "cpu_sweep.json"))
    a = ap.parse_args()
    ln = 1500
    n = a.mib * (1 << 20) // ln
    sample = np.random.default_rng(1).integers(0, 256, n * ln, dtype=np.uint8)
    kind = "reference" if O.ref_available() else "port"
    rows = []
    for osf in ([False, True] if kind == "reference" and O.ref_available(os_flags=True) else [False]):
        for t in (1, 2, 4, 8, 16):
            secs, _ = O.uniform_mt(sample, ln, ln, n, t, kind=kind, os_flags=osf)      # page-in / warm
            reps = max(1, int(a.seconds / max(secs, 1e-3)))
            tot = sum(O.uniform_mt(sample, ln, ln, n, t, kind=kind, os_flags=osf)[0] for _ in range(reps))
            rows.append({"threads": t, "build": "-Os" if osf else "-O3", "GiB_s": round(n * ln * reps / tot / GIB, 2),
                         "passes": reps})
            print(json.dumps(rows[-1]), flush=True)
    cpu = "?"
    try:
        cpu = next(x.split(":", 1)[1].strip() for x in open("/proc/cpuinfo") if x.startswith("model name"))
    except (OSError, StopIteration):
        pass
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"kind": kind, "frames": n, "frame_bytes": ln, "cpu": cpu,
               "usable_cores": len(os.sched_getaffinity(0)), "rows": rows}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
