#!/usr/bin/env python3
"""Interleaved A/B of library builds and launch shapes on one box (bench lines without the CPU
and host legs; every run under its own `timeout`; the first failure ends the script).

  python tools/ab.py --tag T --configs c2,c2v6 --rounds 2 \\
      --variant r04=ablib/libpicocsum_r04.so --variant new= --variant "classic=:--stream 255,0"

A variant is name=[library][:extra bench args]; an empty library is the in-tree one.  Output: gpurun_out/ab_<tag>.txt, one line per run: variant config kernel_avg_us value
mismatches (or '-' with --no-verify)."""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="ab")
    ap.add_argument("--configs", default="c2")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--variant", action="append", default=[])
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, f"ab_{a.tag}.txt")
    variants = []
    for v in a.variant:
        name, rest = v.split("=", 1)
        lib, _, extra = rest.partition(":")
        variants.append((name, lib, shlex.split(extra)))
    with open(path, "w") as log:
        for r in range(a.rounds):
            for cfg in a.configs.split(","):
                for name, lib, extra in variants:
                    env = dict(os.environ)
                    if lib:
                        env["PICO_CSUM_LIB"] = os.path.join(ROOT, lib)
                    else:
                        env.pop("PICO_CSUM_LIB", None)
                    cmd = ["timeout", "-k", "10", "180", sys.executable, os.path.join(ROOT, "bench.py"),
                           "--config", cfg, "--steps", str(a.steps), "--warmup", "10", "--no-cpu", "--no-e2e"]
                    if not a.verify:
                        cmd.append("--no-verify")
                    p = subprocess.run(cmd + extra, env=env, capture_output=True, text=True)
                    if p.returncode != 0:
                        log.write(f"{name} {cfg} FAILED rc={p.returncode}\n{p.stderr[-3000:]}\n")
                        log.flush()
                        print(f"ab: {name} {cfg} failed rc={p.returncode}", flush=True)
                        sys.exit(1)
                    d = json.loads(p.stdout.strip().splitlines()[-1])
                    mm = d.get("verified", {}).get("mismatches", "-")
                    line = f"{name} {cfg} {d['roofline']['kernel_avg_us']} {d['value']} {mm}"
                    log.write(line + "\n")
                    log.flush()
                    print(line, flush=True)


if __name__ == "__main__":
    main()
