#!/usr/bin/env python3
"""Per-wave timeline of the sorted-rounds kernel from the diagnostic build
(picotcp_amd/diag/libpicocsum_stamps.so, `make -C picotcp_amd/csrc diag`): every wave stamps
s_memrealtime (100 MHz) at entry, after phase 1 (descriptors, head windows, parse), after the
rounds and at the end.  Run on a C2 batch (rotating copies, the stamps of the last launch):

    PICO_CSUM_LIB=picotcp_amd/diag/libpicocsum_stamps.so python tools/stamps.py --config c2

Prints the kernel span and, per phase, percentiles over the waves of its start / duration,
plus how much of the span the slowest waves' tail takes.  --config c1stream / c4stream: the
uniform rings' stream waves (csum_uniform_stream_kernel forced on) on C1 / C4 rings -- slots 0 and
3 the entry and end, 1 when the first step's data is in, 2 = 3."""
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
os.environ.setdefault("PICO_CSUM_LIB", os.path.join(ROOT, "picotcp_amd", "diag", "libpicocsum_stamps.so"))
from picotcp_amd import _lib, batch, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c2", "c2tx", "c2v6", "c2raw", "c1stream", "c4stream"])
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--rotate", type=int, default=12)
    ap.add_argument("--wpb", type=int, default=4, help="waves per workgroup of the kernel")
    ap.add_argument("--balanced", action="store_true",
                    help="every group of 64 datagrams the same size multiset (tools/balance_probe.py)")
    a = ap.parse_args()
    lib = _lib.load()
    lib.pico_csum_diag_set_stamps.restype = ctypes.c_int
    lib.pico_csum_diag_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    dev = torch.device("cuda:0")
    n = a.n
    uni = a.config in ("c1stream", "c4stream")
    if a.config == "c4stream":
        n = 1 << 22
    lens = synth.imix_lengths(n, 3) + (20 if a.config == "c2v6" else 0)
    if a.balanced:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from balance_probe import balanced_lengths
        lens = balanced_lengths(n, 3) + (20 if a.config == "c2v6" else 0)
    sets = []
    if uni:           # uniform 1500 B rings on the stream waves (stamps: entry, first step in, end)
        batch.set_uniform_stream(1, 0)
    for r in range(a.rotate if not uni else (a.rotate if n <= 262144 else 2)):
        if uni:
            b = torch.randint(0, 256, (n * 1500,), dtype=torch.uint8, device=dev)
            sets.append((b, None))
            continue
        if a.config == "c2v6":
            buf, net, avail, seeds = synth.ipv6_batch(lens.astype(np.uint32), seed=10 + r, proto=6, eth=True)
            d = batch.desc_to_device(batch.make_desc(net, avail, seeds), dev)
            b = torch.from_numpy(buf).to(dev)
            batch.ipv6_checksum_batch(b, d, n, flags=batch.F_TX | batch.F_WRITE)
        else:
            buf, net, avail = synth.ipv4_batch(lens, seed=10 + r, proto=6, eth=True)
            d = batch.desc_to_device(batch.make_desc(net, avail), dev)
            b = torch.from_numpy(buf).to(dev)
            batch.ipv4_checksum_batch(b, d, n, flags=batch.F_TX | batch.F_WRITE)
        sets.append((b, d))
    waves = -(-n // 64) + 64
    st = torch.zeros(4 * waves, dtype=torch.int64, device=dev)

    def launch(i):
        b, d = sets[i % len(sets)]
        if uni:
            batch.checksum_uniform(b, 1500, 1500, n)
        elif a.config == "c2v6":
            batch.ipv6_checksum_batch(b, d, n)
        elif a.config == "c2raw":
            batch.checksum_batch(b, d, n)
        else:
            batch.ipv4_checksum_batch(b, d, n, flags=batch.F_TX | batch.F_WRITE if a.config == "c2tx" else 0)
    for i in range(30):
        launch(i)
    torch.cuda.synchronize()
    assert lib.pico_csum_diag_set_stamps(ctypes.c_void_p(st.data_ptr()), waves) == 0
    res = []
    for rep in range(5):
        st.zero_()
        torch.cuda.synchronize()
        launch(100 + rep)
        torch.cuda.synchronize()
        t = st.cpu().numpy().reshape(-1, 4)
        wid = np.nonzero(t[:, 0] > 0)[0]
        res.append((t[t[:, 0] > 0], wid))
    lib.pico_csum_diag_set_stamps(ctypes.c_void_p(0), 0)
    out = []
    for t, wid in res:
        t0 = t[:, 0].min()
        rel = (t - t0) * 10.0 / 1000.0          # 100 MHz ticks -> us
        span = rel[:, 3].max()
        q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 99, 100)]
        out.append({"waves": int(t.shape[0]), "span_us": round(float(span), 2),
                    "start_pctl": q(rel[:, 0]), "phase1_end_pctl": q(rel[:, 1]), "rounds_end_pctl": q(rel[:, 2]),
                    "end_pctl": q(rel[:, 3]), "phase1_dur_pctl": q(rel[:, 1] - rel[:, 0]),
                    "rounds_dur_pctl": q(rel[:, 2] - rel[:, 1]), "finish_dur_pctl": q(rel[:, 3] - rel[:, 2]),
                    "waves_done_at_90pct_span": round(float((rel[:, 3] <= 0.9 * span).mean()), 3)})
        # per XCD (workgroups go round-robin over the 8 XCDs; 4 waves a workgroup): medians of the
        # start, the streaming phase and the end, and each XCD's share of the last 5 % of waves
        xcd = (wid // a.wpb) % 8
        late = rel[:, 3] >= np.percentile(rel[:, 3], 95)
        out[-1]["per_xcd"] = [{"xcd": x, "start_med": round(float(np.median(rel[xcd == x, 0])), 2),
                               "rounds_med": round(float(np.median(rel[xcd == x, 2] - rel[xcd == x, 1])), 2),
                               "end_med": round(float(np.median(rel[xcd == x, 3])), 2),
                               "end_max": round(float(rel[xcd == x, 3].max()), 2),
                               "late_share": round(float((late & (xcd == x)).sum() / max(1, late.sum())), 3)}
                              for x in range(8)]
    for o in out:
        print(json.dumps({"config": a.config + ("_balanced" if a.balanced else ""), **o}))


if __name__ == "__main__":
    main()
