#!/usr/bin/env python3
"""FETCH_SIZE calibration for partial-line reads: raw descriptor batches
whose read footprint is known exactly -- `len` bytes at the start of every `stride`-byte slot
(16-byte aligned), over >= 1 GiB of rotated buffers so neither L2 nor the Infinity Cache can
serve a repeat -- run under `rocprofv3 --pmc FETCH_SIZE`, one pattern per process:

    python tools/fetch_calib.py --len 64 --stride 128 --steps 20

Prints one JSON line: pattern, frames, algorithmic bytes per launch (len x n + 16 x n
descriptors + 2 x n results).  FETCH_SIZE (kB) x 1024 / algorithmic bytes then gives the
counter's factor for that access shape (tools/pmc_summary.py)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from picotcp_amd import batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--len", type=int, default=64)
    ap.add_argument("--stride", type=int, default=128)
    ap.add_argument("--frames", type=int, default=262144)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n, ln, st = a.frames, a.len, a.stride
    per = n * st
    rot = max(3, -(-(1 << 30) // per))
    bufs = [torch.randint(0, 256, (per,), dtype=torch.uint8, device=dev) for _ in range(rot)]
    d = batch.desc_to_device(batch.make_desc(np.arange(n, dtype=np.uint64) * st, np.full(n, ln)), dev)
    outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(rot)]
    for i in range(a.steps):
        batch.checksum_batch(bufs[i % rot], d, n, out=outs[i % rot])
    torch.cuda.synchronize()
    print(json.dumps({"pattern": f"len{ln}_stride{st}", "frames": n, "len": ln, "stride": st,
                      "algorithmic_bytes": n * ln + 18 * n, "frame_bytes": n * ln}))


if __name__ == "__main__":
    main()
