#!/usr/bin/env python3
"""Launch-shape sweep in ONE process, variants interleaved over rounds
(cdna_hip_programming.md 5.4 rule 24).  Prints one JSON line per (config, shape)
with the median kernel time and the achieved algorithmic GB/s.

  python tools/sweep.py --config c1 --rounds 5 --shapes 64,2,2,32,1 64,2,1,32,1 ...
  shape = G,CPL,U,FPW,NT[,PIPE]   (NT / PIPE: 1 off, 2 on; G = 1: flat work-list kernel)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from picotcp_amd import batch, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", nargs="*", default=[])
    ap.add_argument("--rotate", type=int, default=12, help="descriptor configs: batch copies rotated "
                    "(12 x ~93 MB >= 1 GiB: the Infinity Cache cannot serve repeats)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    UNI = {"c1": (262144, 1500, 1500), "c3": (262144, 9000, 9000), "c3_64k": (16384, 65536, 65536),
           "c1_1536": (262144, 1500, 1536), "u354": (262144, 354, 354), "u64": (262144, 64, 64),
           "u576": (262144, 576, 576)}
    if a.config in UNI:
        n, ln, stride = UNI[a.config]
        per = (n - 1) * stride + ln
        rot = max(3, -(-(3 << 30) // per) // 2)
        bufs = [torch.randint(0, 256, (per,), dtype=torch.uint8, device=dev) for _ in range(rot)]
        outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(rot)]

        def launch(i):
            batch.checksum_uniform(bufs[i % rot], stride, ln, n, out=outs[i % rot])
        algo = n * ln + 2 * n
    elif a.config == "c1d" or (a.config.startswith("u") and a.config.endswith("d")):
        # uniform frames fed as a descriptor batch (ablation: descriptor kernels vs uniform
        # ones): c1d = 256K x 1500 B, u<LEN>d = 256K x LEN bytes
        n, ln = 262144, 1500 if a.config == "c1d" else int(a.config[1:-1])
        rot = max(3, -(-(1 << 30) // (n * ln)))
        bufs = [torch.randint(0, 256, (n * ln,), dtype=torch.uint8, device=dev) for _ in range(rot)]
        d_desc = batch.desc_to_device(batch.make_desc(np.arange(n, dtype=np.uint64) * ln, np.full(n, ln)), dev)
        outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(rot)]

        def launch(i):
            batch.checksum_batch(bufs[i % rot], d_desc, n, out=outs[i % rot])
        algo = n * ln + 18 * n
    elif a.config == "c2v6":
        n = 262144
        lens = (synth.imix_lengths(n, 3) + 20).astype(np.uint32)
        rot = a.rotate
        sets = []
        for r in range(rot):
            buf, net, avail, seeds = synth.ipv6_batch(lens, seed=10 + r, proto=6, eth=True)
            d_buf = torch.from_numpy(buf).to(dev)
            d_desc = batch.desc_to_device(batch.make_desc(net, avail, seeds), dev)
            batch.ipv6_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
            sets.append((d_buf, d_desc))

        def launch(i):
            b, d = sets[i % rot]
            batch.ipv6_checksum_batch(b, d, n)
        algo = int(lens.sum()) + 19 * n
    elif a.config == "c2eth":
        # the C2 datagrams through the Ethernet front end (descriptors -> frame start)
        n = 262144
        lens = synth.imix_lengths(n, 3)
        rot = a.rotate
        sets = []
        for r in range(rot):
            buf, net, avail = synth.ipv4_batch(lens, seed=10 + r, proto=6, eth=True)
            d_buf = torch.from_numpy(buf).to(dev)
            d_desc = batch.desc_to_device(batch.make_desc(net - np.uint64(14), avail + 14), dev)
            batch.eth_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
            sets.append((d_buf, d_desc))
        o3 = [(torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
               torch.empty(n, dtype=torch.uint8, device=dev)) for r in range(rot)]

        def launch(i):
            b, d = sets[i % rot]
            batch.eth_checksum_batch(b, d, n, out=o3[i % rot])
        algo = int(lens.sum()) + 14 * n + 16 * n + 5 * n
    elif a.config in ("c2raw", "c2", "c2tx", "c2txnw"):
        n = 262144
        lens = synth.imix_lengths(n, 3)
        rot = a.rotate
        sets = []
        for r in range(rot):
            buf, net, avail = synth.ipv4_batch(lens, seed=10 + r, proto=6, eth=True)
            d_buf = torch.from_numpy(buf).to(dev)
            d_desc = batch.desc_to_device(batch.make_desc(net, avail), dev)
            batch.ipv4_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
            sets.append((d_buf, d_desc))
        outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(rot)]
        if a.config == "c2raw":
            def launch(i):
                b, d = sets[i % rot]
                batch.checksum_batch(b, d, n, out=outs[i % rot])
        else:
            fl = {"c2": 0, "c2tx": batch.F_TX | batch.F_WRITE, "c2txnw": batch.F_TX}[a.config]
            o3 = [(outs[r], torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.uint8, device=dev))
                  for r in range(rot)]

            def launch(i):
                b, d = sets[i % rot]
                batch.ipv4_checksum_batch(b, d, n, flags=fl, out=o3[i % rot])
        algo = int(lens.sum()) + 16 * n + (2 if a.config == "c2raw" else 5) * n
    else:
        raise SystemExit("unknown config")

    shapes = [tuple(int(x) for x in s.split(",")) for s in a.shapes] or [(0, 0, 0, 0, 0)]
    times = {s: [] for s in shapes}
    stream = torch.cuda.current_stream()
    for rnd in range(a.rounds):
        for s in shapes:
            g, c, u, f, nt = s[:5]
            batch.set_launch_override(g, c, f, u, nt, s[5] if len(s) > 5 else 0)
            for i in range(3):
                launch(i)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
            for i in range(a.iters):
                evs[i][0].record(stream)
                launch(i)
                evs[i][1].record(stream)
            torch.cuda.synchronize()
            times[s].append(float(np.median([x.elapsed_time(y) for x, y in evs])))
    batch.set_launch_override(0)
    for s in shapes:
        t = float(np.median(times[s]))
        print(json.dumps({"config": a.config, "shape": "auto" if s[0] == 0 else ",".join(map(str, s)),
                          "us": round(t * 1e3, 2), "us_min_round": round(min(times[s]) * 1e3, 2),
                          "GBs": round(algo / (t / 1e3) / 1e9, 1), "frac": round(algo / (t / 1e3) / 8e12, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
