#!/usr/bin/env python3
"""Measurement aid: the bare gather of bench.py's reassembly batch (c3_reasm / c3_reasm6 /
c3_reasm_il layout) -- tools/gather_ceiling.hip copies every fragment's payload to its place in the
output, nothing parsed or summed -- timed with HIP events beside the reassembly kernel itself on the
same batch, interleaved, and the device's sequential copy of the same bytes.  The practical ceiling
the reassembly kernel is priced against; bare_gather has the reassembly kernel's
shape (one wave per datagram, two fragments a step), the other bare gathers other grid shapes.

  hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/gather_ceiling.hip -o tools/bin/libgather_ceiling.so
  python tools/gather_ceiling.py [--v6] [--interleave] [--reps 50]
"""
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
import bench  # noqa: E402
from picotcp_amd import batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--v6", action="store_true")
    ap.add_argument("--interleave", action="store_true")
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rotate", type=int, default=4)
    ap.add_argument("--reasm-flat", type=int, default=0, help="pico_csum_set_reasm_flat mode for the reassembly")
    ap.add_argument("--only-reasm", action="store_true", help="time the reassembly alone")
    a = ap.parse_args()
    batch.set_reasm_flat(a.reasm_flat)
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "libgather_ceiling.so"))
    lib.seq_copy_launch.restype = ctypes.c_int
    lib.seq_copy_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_void_p]
    lib.gather_ceiling_launch.restype = ctypes.c_int
    lib.gather_ceiling_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 4 + \
        [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    tl = 64512
    hl = 48 if a.v6 else 20
    H = 40 if a.v6 else 20
    fr = bench.FRAG6 if a.v6 else bench.FRAG
    sets = []
    for r in range(a.rotate):
        st = bench.make_frag(a.n, tl, dev, 100 + r, v6=a.v6, interleave=a.interleave)
        buf, d_desc, d_grp, out, d_od, nfr, payload = st
        desc = d_desc.cpu().numpy().view(batch.DESC_DTYPE)
        od = d_od.cpu().numpy().view(batch.DESC_DTYPE)
        grp = d_grp.cpu().numpy().view(np.uint32).reshape(-1, 2)
        nf = int(grp[0, 1])
        k = np.tile(np.arange(nf), a.n)
        g = np.repeat(np.arange(a.n), nf)
        f_src = desc["off"].astype(np.uint64) + np.uint64(hl)
        f_len = (desc["len"].astype(np.int64) - hl).astype(np.uint32)
        f_dst = od["off"][g].astype(np.uint64) + np.uint64(H) + (k * fr).astype(np.uint64)
        t = [torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x.view(np.int32)).to(dev)
             for x in (f_src, f_dst, f_len)]
        sets.append((st, t, d_grp))
    s = torch.cuda.current_stream(dev)

    def gather(mode):
        def f(i):
            (buf, d_desc, d_grp, out, d_od, nfr, payload), (fs, fd, fl), gr = sets[i % a.rotate]
            rc = lib.gather_ceiling_launch(mode, buf.data_ptr(), buf.numel(), fs.data_ptr(), fd.data_ptr(), fl.data_ptr(),
                                           gr.data_ptr(), a.n, nfr, out.data_ptr(), out.numel(),
                                           ctypes.c_void_p(s.cuda_stream))
            assert rc == 0
        return f

    def reasm(i):
        (buf, d_desc, d_grp, out, d_od, nfr, payload), _, _ = sets[i % a.rotate]
        fn = batch.ipv6_reassemble_batch if a.v6 else batch.ipv4_reassemble_batch
        fn(buf, d_desc, nfr, d_grp, out, d_od)

    def copy(i):
        (buf, d_desc, d_grp, out, d_od, nfr, payload), _, _ = sets[i % a.rotate]
        out[:payload].copy_(buf[:payload])

    def seq_copy(var, u, blocks):             # the hand-written sequential copy (bench.copy_ceiling)
        def f(i):
            (buf, d_desc, d_grp, out, d_od, nfr, payload), _, _ = sets[i % a.rotate]
            assert lib.seq_copy_launch(var, u, blocks, out.data_ptr(), buf.data_ptr(), payload & ~15,
                                       ctypes.c_void_p(s.cuda_stream)) == 0
        return f

    def timed(f):
        for i in range(5):
            f(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record(s)
        for i in range(a.reps):
            f(i)
        e1.record(s)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) * 1e3 / a.reps

    payload = sets[0][0][6]
    res = {}
    fns = (("reassemble", reasm),) if a.only_reasm else (
        ("reassemble", reasm), ("bare_gather", gather(0)), ("bare_gather_4frag_steps", gather(1)),
        ("bare_gather_4waves", gather(2)), ("bare_gather_flat", gather(3)), ("sequential_copy_torch", copy),
        ("sequential_copy_nt", seq_copy(0, 4, 0)), ("sequential_copy_cached", seq_copy(1, 4, 0)),
        ("sequential_copy_nt_grid", seq_copy(0, 4, 8192)), ("sequential_copy_unaligned_src", seq_copy(3, 4, 0)),
        ("sequential_copy_unaligned_src_nt", seq_copy(4, 4, 0)),
        ("sequential_copy_unaligned_src_nt_stores", seq_copy(5, 4, 0)),
        ("sequential_copy_aligned_nt_shifted", seq_copy(6, 4, 0)))
    if not a.only_reasm:                      # variant 6 moves the same bytes as variant 3
        (buf, d_desc, d_grp, out, d_od, nfr, payload), _, _ = sets[0]
        n = (payload & ~15) - 16
        seq_copy(3, 4, 0)(0)
        ref = out[:n].clone()
        out[:n].zero_()
        seq_copy(6, 4, 0)(0)
        torch.cuda.synchronize(dev)
        assert torch.equal(ref, out[:n]), "seq_copy variant 6 differs from variant 3"
    for rnd in range(3):
        for name, f in fns:
            res.setdefault(name, []).append(timed(f))
    out = {"layout": ("ipv6" if a.v6 else "ipv4") + (" interleaved" if a.interleave else " datagram-major"),
           "datagrams": a.n, "payload_bytes": payload, "reasm_flat": a.reasm_flat}
    for name, v in res.items():
        us = float(np.median(v))
        out[name + "_us"] = round(us, 2)
        out[name + "_TBs_rw"] = round(2 * payload / us / 1e6, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
