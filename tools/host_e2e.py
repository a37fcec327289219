#!/usr/bin/env python3
"""Host-to-host rate of the host-resident fused IPv4 batch (pico_ipv4_checksum_batch_host) on the
C2 burst (pinned) for several staging sizes, staged and / or read in place, interleaved in one
process (A/B of the chunking).

  python tools/host_e2e.py [--stagings 8 16 32 64] [--rounds 3] [--mode staged|in_place|both]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from picotcp_amd import batch, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stagings", type=int, nargs="*", default=[8, 16, 32, 64])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--mode", default="staged", choices=["staged", "in_place", "both"],
                    help="the staged path, the in-place path (the burst is pinned), or both interleaved")
    a = ap.parse_args()
    n = 262144
    lens = synth.imix_lengths(n, 3)
    buf, net, avail = synth.ipv4_batch(lens, seed=10, proto=6, eth=True)
    desc = batch.make_desc(net, avail)
    pinned = torch.from_numpy(buf).pin_memory().numpy()
    nbytes = int(desc["len"].astype(np.int64).sum())
    modes = {"in_place": True, "staged": False} if a.mode == "both" else {a.mode: a.mode == "in_place"}
    res = {(s, m): [] for s in a.stagings for m in modes}
    hbs = {s: batch.HostBatch(torch.cuda.current_device(), staging_bytes=s << 20) for s in a.stagings}
    try:
        for _ in range(a.rounds):
            for s in a.stagings:
                for m, on in modes.items():
                    hb = hbs[s]
                    batch.set_host_in_place(on)
                    hb.ipv4_checksum_batch(pinned, desc)
                    t0 = time.perf_counter()
                    for _ in range(a.reps):
                        hb.ipv4_checksum_batch(pinned, desc)
                    res[(s, m)].append(nbytes / ((time.perf_counter() - t0) / a.reps) / (1 << 30))
    finally:
        batch.set_host_in_place(True)
        for hb in hbs.values():
            hb.close()
    for (s, m), v in res.items():
        print(json.dumps({"staging_MiB": s, "path": m, "GiBs_median": round(float(np.median(v)), 2),
                          "GiBs_all": [round(x, 2) for x in v]}), flush=True)


if __name__ == "__main__":
    main()
