#!/usr/bin/env python3
"""Golden forwarding-step sequence from the reference's own pico_ipv4_pre_forward_checks.

Run here (where /root/reference exists):
    make -C oracle refrx && python tests/golden/make_ref_fwd.py

oracle/_ref/libref_rx.so is the reference stack compiled unmodified (oracle/Makefile `refrx`);
its driver's rr_forward (oracle/ref_rx_driver.c) runs the static pico_ipv4_pre_forward_checks
(modules/pico_ipv4.c:1535-1574, reached through oracle/ref_rx_wrap.c unit 1) on one datagram:
  * hdr->ttl - 1, discarded when it reaches 0 (:1548-1553);
  * hdr->crc++ (:1556);
  * discarded when the source is one of the stack's own link addresses (pico_ipv4_link_get, :1559);
  * discarded when (src, id, dst, proto) equals the last datagram that reached this check, else
    that tuple becomes the last one (:1562-1571) -- static state, zero at start, so a first
    datagram with an all-zero tuple is a duplicate.
The datagrams are fed IN ORDER through a fresh library copy (the reference's initial state), so
the fixture is one sequence: a batch implementation must carry the last-forwarded tuple from one
batch to the next to reproduce it.  Cases: TTL 0 / 1 / 2 / 255 and random, back-to-back repeats
of one tuple, tuples interleaved from small pools (so repeats are separated by other datagrams,
expired ones and local sources), local sources (three links), options (IHL > 5), odd offsets.
Datagrams shorter than 20 bytes are added without a reference call (the stack never forwards
them): their expected bytes are the input and their verdict MALFORMED (restatement only).

Output (data only): ref_fwd_cases.npz
  buf uint8[], off uint64[n], avail uint32[n], want uint8[] (buf after the steps, in order),
  ret int32[n] (rr_forward: 0 forwarded, 1 expired, 2 local, 3 duplicate; -9 not called),
  verdict uint8[n] (expected batch verdict), local uint32[k] (link addresses as stored)
"""
from __future__ import annotations

import ctypes
import os
import shutil
import sys
import tempfile

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

OUT = os.path.dirname(os.path.abspath(__file__))
REF_RX = os.path.join(ROOT, "oracle", "_ref", "libref_rx.so")
V_ACCEPT, V_MALFORMED, V_EXPIRED, V_LOCAL_SRC, V_DUPLICATE = 1, 8, 16, 32, 64
RET_VERDICT = {0: V_ACCEPT, 1: V_EXPIRED, 2: V_LOCAL_SRC, 3: V_DUPLICATE}
LOCAL = [bytes([10, 0, 0, 1]), bytes([192, 168, 1, 1]), bytes([172, 16, 5, 9])]


def ref_lib():
    """A private copy of libref_rx.so: its pre-forward state starts at the reference's zeros."""
    tmp = tempfile.NamedTemporaryFile(suffix=".so", delete=False)
    tmp.close()
    shutil.copyfile(REF_RX, tmp.name)
    R = ctypes.CDLL(tmp.name)
    os.unlink(tmp.name)
    R.rr_init.restype = ctypes.c_int
    R.rr_ipv4_link.restype = ctypes.c_int
    R.rr_ipv4_link.argtypes = [ctypes.c_uint32]
    R.rr_forward.restype = ctypes.c_int
    R.rr_forward.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    if R.rr_init() != 0:
        raise RuntimeError("rr_init failed")
    for a in LOCAL:
        if R.rr_ipv4_link(int.from_bytes(a, "little")) != 0:
            raise RuntimeError("rr_ipv4_link failed")
    return R


def sequence(seed: int = 11, n: int = 6000):
    """The datagram headers (+ a few payload bytes) of the sequence, in order."""
    rng = np.random.default_rng(seed)
    srcs = [bytes([10, 1, 2, 3]), bytes([10, 9, 9, 9]), bytes([198, 51, 100, 7]), bytes([0, 0, 0, 0]),
            bytes([10, 1, 2, 4])] + LOCAL[:1]
    dsts = [bytes([10, 4, 4, 4]), bytes([203, 0, 113, 5]), bytes([0, 0, 0, 0]), bytes([8, 8, 8, 8])]
    ids = [0, 0x1234, 0xFFFF]
    protos = [6, 17, 1, 0]
    out = []
    # the all-zero tuple first: a duplicate of the reference's initial state
    out.append(dict(src=bytes(4), dst=bytes(4), ident=0, proto=0, ttl=64, ihl=5, extra=0))
    tup = None
    while len(out) < n:
        mode = rng.integers(0, 10)
        if tup is None or mode < 6:                  # a fresh tuple from the pools
            tup = (srcs[rng.integers(0, len(srcs))], dsts[rng.integers(0, len(dsts))],
                   ids[rng.integers(0, len(ids))] if rng.random() < 0.7 else int(rng.integers(0, 1 << 16)),
                   protos[rng.integers(0, len(protos))])
        reps = 1 if mode < 7 else int(rng.integers(2, 5))    # back-to-back repeats
        for _ in range(reps):
            r = rng.random()
            ttl = int(rng.choice([0, 1, 2, 255])) if r < 0.25 else int(rng.integers(0, 256))
            if rng.random() < 0.05:                   # a local source in between
                s = LOCAL[rng.integers(0, len(LOCAL))]
                out.append(dict(src=s, dst=tup[1], ident=tup[2], proto=tup[3], ttl=ttl, ihl=5, extra=0))
            out.append(dict(src=tup[0], dst=tup[1], ident=tup[2], proto=tup[3], ttl=ttl,
                            ihl=int(rng.choice([5, 5, 5, 6, 15])), extra=int(rng.integers(0, 40))))
    return out[:n]


def main() -> None:
    R = ref_lib()
    rng = np.random.default_rng(5)
    rows = sequence()
    bufs, offs, avails = [], [], []
    pos = 0
    for k, d in enumerate(rows):
        hl = 4 * d["ihl"]
        ln = hl + d["extra"]
        b = rng.integers(0, 256, ln, dtype=np.uint8)
        b[0] = 0x40 | d["ihl"]
        b[2], b[3] = ln >> 8, ln & 0xFF
        b[4], b[5] = d["ident"] >> 8, d["ident"] & 0xFF
        b[8] = d["ttl"]
        b[9] = d["proto"]
        b[12:16] = list(d["src"])
        b[16:20] = list(d["dst"])
        if k % 97 == 50:                             # shorter than an IPv4 header: never forwarded
            b = b[:int(rng.integers(0, 20))]
        gap = int(rng.integers(0, 4))                # odd offsets too
        pos += gap
        offs.append(pos)
        avails.append(b.size)
        bufs.append((pos, b))
        pos += b.size
    buf = np.zeros(pos + 16, np.uint8)
    for o, b in bufs:
        buf[o:o + b.size] = b
    want = buf.copy()
    ret = np.full(len(rows), -9, np.int32)
    verdict = np.zeros(len(rows), np.uint8)
    for i, (o, ln) in enumerate(zip(offs, avails)):
        if ln < 20:
            verdict[i] = V_MALFORMED
            continue
        d = np.ascontiguousarray(want[o:o + ln])
        ret[i] = R.rr_forward(d.ctypes.data, ln)
        if ret[i] < 0:
            raise RuntimeError(f"rr_forward failed on row {i}")
        want[o:o + ln] = d
        verdict[i] = RET_VERDICT[int(ret[i])]
    local = np.array([int.from_bytes(a, "little") for a in LOCAL], np.uint32)
    np.savez_compressed(os.path.join(OUT, "ref_fwd_cases.npz"), buf=buf, off=np.array(offs, np.uint64),
                        avail=np.array(avails, np.uint32), want=want, ret=ret, verdict=verdict, local=local)
    u, c = np.unique(verdict, return_counts=True)
    print("ref_fwd_cases.npz:", len(rows), "datagrams;", dict(zip(u.tolist(), c.tolist())))


if __name__ == "__main__":
    main()
