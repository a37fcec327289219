#!/usr/bin/env python3
"""How much of C2's launch is the per-wave byte spread?  (A measurement aid, not the product.)

Times the fused IPv4 RX batch (K4s MODE 1, 64 datagrams a wave) on two layouts of the same
simple-IMIX mix, interleaved in one process:
  imix      -- the bench's C2 batch: sizes in seeded random order, so a wave's 64 datagrams carry
               p1 14.9 KB .. p99 30.5 KB;
  balanced  -- every aligned group of 64 datagrams holds the same multiset (37 x 64 B, 21 x 576 B,
               6 x 1500 B, then 38 / 21 / 5: 23 464 / 22 028 B), shuffled inside the group: the
               byte spread across waves is +-3 %, total bytes within 0.3 % of imix.
The gap between the two per byte bounds what any byte-balanced partition can win on C2.
  prepass   -- the device pre-pass such a partition needs inside the step (tools/c2_prepass.hip:
               one lane per descriptor writes each wave's first datagram at equal-byte boundaries),
               alone on the imix batch;
  prepass+imix -- that pre-pass followed by the C2 kernel, each step: the partition's entry fee.
Every variant is K steps captured as one HIP graph and replayed (as bench.py times), interleaved.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/c2_prepass.hip -o tools/bin/libc2_prepass.so
    python tools/balance_probe.py [--rounds 5] [--steps 20]"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from picotcp_amd import batch, synth  # noqa: E402


def balanced_lengths(n: int, seed: int) -> np.ndarray:
    groups = []
    rng = np.random.default_rng(seed)
    for g in range(-(-n // 64)):
        a, b, c = (37, 21, 6) if g % 2 == 0 else (38, 21, 5)
        grp = np.array([64] * a + [576] * b + [1500] * c, dtype=np.uint32)
        rng.shuffle(grp)
        groups.append(grp)
    return np.concatenate(groups)[:n]


def make(lens, dev, seed):
    buf, net, avail = synth.ipv4_batch(lens, seed=seed, proto=6, eth=True)
    d_buf = torch.from_numpy(buf).to(dev)
    d_desc = batch.desc_to_device(batch.make_desc(net, avail), dev)
    batch.ipv4_checksum_batch(d_buf, d_desc, lens.size, flags=batch.F_TX | batch.F_WRITE)
    return d_buf, d_desc, int(lens.sum()) + 14 * lens.size


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rotate", type=int, default=12)
    ap.add_argument("--waves", type=int, default=4096, help="W of the pre-pass (equal-byte spans)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n = a.n
    pre = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libc2_prepass.so"))
    pre.c2_prepass_launch.restype = ctypes.c_int
    pre.c2_prepass_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                      ctypes.c_void_p]
    sets = {
        "imix": [make(synth.imix_lengths(n, 500 + 13 * i), dev, 501 + 13 * i) for i in range(a.rotate)],
        "balanced": [make(balanced_lengths(n, 700 + i), dev, 701 + 13 * i) for i in range(a.rotate)],
    }
    torch.cuda.synchronize()
    for k, v in sets.items():
        o = batch.ipv4_checksum_batch(v[0][0], v[0][1], n)
        torch.cuda.synchronize()
        assert bool((o[2] == 1).all()), f"{k}: not every datagram accepted"
    outs = {k: batch.ipv4_checksum_batch(v[0][0], v[0][1], n) for k, v in sets.items()}
    starts = torch.zeros(a.waves + 1, dtype=torch.int32, device=dev)

    def prepass(s):
        h = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        assert pre.c2_prepass_launch(ctypes.c_void_p(s[1].data_ptr()), n, a.waves,
                                     ctypes.c_void_p(starts.data_ptr()), h) == 0

    # the pre-pass against numpy on one batch
    s0 = sets["imix"][0]
    prepass(s0)
    torch.cuda.synchronize()
    d = s0[1].cpu().numpy().view(batch.DESC_DTYPE)
    pos = (d["off"] - d["off"][0]).astype(np.int64)
    span = int(d["off"][-1] + d["len"][-1] - d["off"][0])
    B = -(-span // a.waves)
    want = np.searchsorted(pos, np.arange(a.waves + 1, dtype=np.int64) * B, side="left")
    got = starts.cpu().numpy()
    assert np.array_equal(got, want), "pre-pass disagrees with numpy"
    cnt = np.diff(want)
    spread = {"datagrams_per_wave_pctl": [int(np.percentile(cnt, p)) for p in (0, 1, 50, 99, 100)],
              "waves_over_64": int((cnt > 64).sum())}

    variants = {
        "imix": (sets["imix"], lambda s, o: batch.ipv4_checksum_batch(s[0], s[1], n, out=o)),
        "balanced": (sets["balanced"], lambda s, o: batch.ipv4_checksum_batch(s[0], s[1], n, out=o)),
        "prepass": (sets["imix"], lambda s, o: prepass(s)),
        "prepass+imix": (sets["imix"], lambda s, o: (prepass(s), batch.ipv4_checksum_batch(s[0], s[1], n, out=o))),
    }
    graphs = {}
    cur = torch.cuda.current_stream()
    for k, (v, fn) in variants.items():
        o = outs["balanced" if k == "balanced" else "imix"]
        for i in range(3):
            fn(v[i % len(v)], o)
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(cur)
        with torch.cuda.stream(cap):
            with torch.cuda.graph(g, stream=cap):
                for i in range(a.steps):
                    fn(v[i % len(v)], o)
        cur.wait_stream(cap)
        g.replay()
        torch.cuda.synchronize()
        graphs[k] = g
    res = {k: [] for k in variants}
    for r in range(a.rounds):
        for k, g in graphs.items():
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000.0 / a.steps
            v = variants[k][0]
            nbytes = sum(s[2] for s in v) / len(v)
            res[k].append({"us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1), "bytes": int(nbytes)})
    # the C2 outputs after the replays still verify (every datagram accepted)
    for k in ("imix", "balanced"):
        assert bool((outs[k][2] == 1).all()), f"{k}: verdicts changed"
    print(json.dumps({"prepass_check": "equal to numpy searchsorted", "W": a.waves, "B": B, **spread}))
    for k, v in res.items():
        print(json.dumps({"variant": k, "rounds": v,
                          "median_us": float(np.median([x["us"] for x in v])),
                          "median_GBps": float(np.median([x["GBps"] for x in v]))}))


if __name__ == "__main__":
    main()
