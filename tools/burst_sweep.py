#!/usr/bin/env python3
"""Launch shapes at realistic burst sizes: per batch size n (1K .. 256K
frames) and per candidate shape, the median launch time (HIP events over `iters` launches, 5
interleaved rounds in ONE process) and the achieved algorithmic bandwidth; `auto` is the
library's own choice (pick_shape / pick_fpw in pico_csum.c).

  python tools/burst_sweep.py --config c2 --sizes 1024 4096 16384 65536 262144
  config: c2 (IMIX IPv4/TCP fused RX, descriptors) | u1500 (uniform 1500 B ring)

Buffers rotate over >= 256 MiB (at most 2048 copies) so repeats do not hit L2; small bursts may
still partly hit the 256 MiB Infinity Cache, as a freshly DMA'd burst would not.
The `iters` launches are captured in one HIP graph (torch.cuda.CUDAGraph over the library's own
launches on the capturing stream) and the replay is timed: at 1K-16K frames the Python launch
path would otherwise be what is measured.  Prints one JSON line per (n, shape)."""
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

# shapes: (group, cpl, fpw, unroll, nt, pipeline) for set_launch_override; fpw 0 = scaled by n below
C2_SHAPES = {"auto": None, "fpw4": (2, 8, 4, 1, 2), "fpw8": (2, 8, 8, 1, 2), "fpw16": (2, 8, 16, 1, 2),
             "fpw32": (2, 8, 32, 1, 2), "fpw64": (2, 8, 64, 1, 2)}
U_SHAPES = {"auto": None, "g16c8f4": (16, 8, 4, 1, 2, 2),
            "g16c8f8": (16, 8, 8, 1, 2, 2), "g16c8f16": (16, 8, 16, 1, 2, 2), "g16c8f32": (16, 8, 32, 1, 2, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--sizes", nargs="*", type=int, default=[1024, 4096, 16384, 65536, 262144])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for n in a.sizes:
        if a.config == "c2":
            lens = synth.imix_lengths(n, 3)
            buf, net, avail = synth.ipv4_batch(lens, seed=10, proto=6, eth=True)
            per = buf.size
            rot = int(min(2048, max(3, -(-(256 << 20) // per))))
            d_desc = batch.desc_to_device(batch.make_desc(net, avail), dev)
            base = torch.from_numpy(buf).to(dev)
            batch.ipv4_checksum_batch(base, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
            bufs = [base] + [base.clone() for _ in range(rot - 1)]
            outs = (torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
                    torch.empty(n, dtype=torch.uint8, device=dev))

            def launch(i):
                batch.ipv4_checksum_batch(bufs[i % rot], d_desc, n, out=outs)
            algo = int(lens.sum()) + 21 * n
            shapes = C2_SHAPES
        else:
            ln = 1500
            per = n * ln
            rot = int(min(2048, max(3, -(-(256 << 20) // per))))
            bufs = [torch.randint(0, 256, (per,), dtype=torch.uint8, device=dev) for _ in range(rot)]
            out = torch.empty(n, dtype=torch.int16, device=dev)

            def launch(i):
                batch.checksum_uniform(bufs[i % rot], ln, ln, n, out=out)
            algo = per + 2 * n
            shapes = U_SHAPES
        times = {k: [] for k in shapes}
        for _ in range(a.rounds):
            for k, sh in shapes.items():
                if sh is None:
                    batch.set_launch_override(0)
                else:
                    try:
                        batch.set_launch_override(*sh)
                    except Exception:
                        continue
                for i in range(5):
                    launch(i)
                torch.cuda.synchronize()
                # the launches captured in a HIP graph: replay measures the GPU, not the Python
                # launch path (small bursts are launch-bound otherwise)
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        for i in range(a.iters):
                            launch(i)
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) / a.iters * 1e3)
                del g
        batch.set_launch_override(0)
        for k, v in times.items():
            if not v:
                continue
            us = float(np.median(v))
            print(json.dumps({"config": a.config, "n": n, "shape": k, "us": round(us, 2),
                              "GBs": round(algo / us / 1e3, 1), "frac": round(algo / us / 1e3 / 8000, 4)}), flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
