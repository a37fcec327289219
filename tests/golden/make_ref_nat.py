#!/usr/bin/env python3
"""Golden NAT rewrites from the reference's own pico_nat.c.

Run here (where /root/reference exists):
    make -C oracle refrx && python tests/golden/make_ref_nat.py

oracle/_ref/libref_rx.so is the reference stack compiled unmodified (oracle/Makefile `refrx`, now
with PICO_SUPPORT_NAT and modules/pico_nat.c); its driver's rr_nat (oracle/ref_rx_driver.c) runs
pico_ipv4_nat_outbound / pico_ipv4_nat_inbound (modules/pico_nat.c:424-545) on one datagram as
pico_ipv4_process_in leaves it, NAT enabled on the link 198.51.100.1.  The cases:
  * outbound: TCP / UDP / ICMPv4 / GRE datagrams from 10.x hosts, with options or not, the
    transport checksum valid, corrupted or (UDP) zero -- the reference's tuple table picks the
    NAT port (pico_rand), read back from its output;
  * inbound: replies to the NAT address on a port of an earlier outbound tuple (translated back)
    or on a port no tuple holds (untouched, the lookup fails: -1).
For every case the fixture keeps the datagram before, the reference's bytes after, its return
value and the record a host would hand the batch (addr / port the reference wrote; dir 0 where
it returned -1 on a TCP / UDP datagram: no tuple).  Fragments and infeasible lengths are added
without a reference call (the stack never hands them to NAT: pico_ipv4.c:446-455, :405-408):
their expected bytes are the input, their verdicts FRAG / MALFORMED ("parity unpinned" there,
restatement only).

Output (data only): ref_nat_cases.npz
  buf uint8[], off uint64[n], avail uint32[n], nat (addr u32, port u16, dir u8, 0) [n],
  want uint8[] (buf after NAT), ret int32[n] (-9: not called), verdict uint8[n] (expected)
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF_RX = os.path.join(ROOT, "oracle", "_ref", "libref_rx.so")
NAT_ADDR = bytes([198, 51, 100, 1])
V_ACCEPT, V_MALFORMED, V_FRAG, V_UNTOUCHED = 1, 8, 16, 32


def ref_lib():
    """A private copy of libref_rx.so (its own stack state: the NAT link and tuples stay out of
    the other fixtures' live re-runs in the same process)."""
    import shutil
    import tempfile
    tmp = tempfile.NamedTemporaryFile(suffix=".so", delete=False)
    tmp.close()
    shutil.copyfile(REF_RX, tmp.name)
    R = ctypes.CDLL(tmp.name)
    os.unlink(tmp.name)
    R.rr_init.restype = ctypes.c_int
    R.rr_nat.restype = ctypes.c_int
    R.rr_nat.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    if R.rr_init() != 0:
        raise RuntimeError("rr_init failed")
    return R


def _sum(b: np.ndarray, s: int = 0) -> int:
    b = np.asarray(b, dtype=np.uint32)
    even = b[0::2].sum()
    odd = b[1::2].sum() if b.size > 1 else 0
    return (s + int(even) + (int(odd) << 8)) & 0xFFFFFFFF   # pico_checksum_adder (LE words)


def _fin(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def datagram(rng, proto, tl, src, dst, sport, dport, opts=0, l4="valid", frag=0x4000):
    hl = 20 + 4 * opts
    h = np.zeros(hl, np.uint8)
    h[0] = 0x40 | (5 + opts)
    tot = hl + tl
    h[2], h[3] = tot >> 8, tot & 0xFF
    h[4], h[5] = rng.integers(256), rng.integers(256)
    h[6], h[7] = frag >> 8, frag & 0xFF
    h[8], h[9] = 64, proto
    h[12:16] = np.frombuffer(src, np.uint8)
    h[16:20] = np.frombuffer(dst, np.uint8)
    if opts:
        h[20:] = rng.integers(0, 256, 4 * opts)
    t = rng.integers(0, 256, tl).astype(np.uint8)
    if proto in (6, 17) and tl >= 4:
        t[0], t[1], t[2], t[3] = sport >> 8, sport & 0xFF, dport >> 8, dport & 0xFF
    crc_at = {6: 16, 17: 6, 1: 2}.get(proto)
    if proto == 6 and tl >= 20:
        t[12] = 0x50
        t[13] = 0x10
    if proto == 17 and tl >= 8:
        t[4], t[5] = tl >> 8, tl & 0xFF
    if crc_at is not None and tl >= crc_at + 2:
        t[crc_at] = t[crc_at + 1] = 0
        if l4 != "zero":
            ph = 0 if proto == 1 else _sum(np.frombuffer(bytes(h[12:20]) + bytes([0, proto, tl >> 8, tl & 0xFF]),
                                                        np.uint8))
            c = _fin(_sum(t, ph))
            if l4 == "bad":
                c ^= 1 + int(rng.integers(0xFFFE))
            t[crc_at], t[crc_at + 1] = c >> 8, c & 0xFF
    c = _fin(_sum(h))
    h[10], h[11] = c >> 8, c & 0xFF
    return np.concatenate([h, t])


def main() -> None:
    rng = np.random.default_rng(0x4A7)
    R = ref_lib()
    nat_addr = int.from_bytes(NAT_ADDR, "little")
    frames, recs, wants, rets, verdicts = [], [], [], [], []
    tuples = []                                  # (proto, remote, nat_port) of translated outbound TCP / UDP

    def add(d, rec, want, ret, v):
        frames.append(d)
        recs.append(rec)
        wants.append(want)
        rets.append(ret)
        verdicts.append(v)

    for k in range(700):
        proto = [6, 6, 17, 17, 1, 47][k % 6]
        tl = int(rng.integers(20 if proto == 6 else 8, 700))
        l4 = ["valid", "valid", "bad", "zero"][int(rng.integers(4))] if proto == 17 else \
            ["valid", "valid", "bad"][int(rng.integers(3))]
        src = bytes([10, 0, int(rng.integers(4)), int(rng.integers(1, 255))])
        dst = bytes([203, 0, 113, int(rng.integers(1, 255))])
        sport, dport = int(rng.integers(1024, 65536)), int(rng.choice([80, 443, 53, 8080, 5000]))
        d = datagram(rng, proto, tl, src, dst, sport, dport, opts=int(rng.integers(3)) if k % 5 == 0 else 0, l4=l4)
        out = d.copy()
        r = R.rr_nat(1, out.ctypes.data, out.size, nat_addr)
        rec = (0, 0, 0)
        if r == 0:
            hl = 20 + 4 * ((out[0] & 0x0F) - 5)
            port = int.from_bytes(bytes(out[hl:hl + 2]), "little") if proto in (6, 17) else 0
            rec = (int.from_bytes(bytes(out[12:16]), "little") if proto in (6, 17) else 0, port, 1)
            if proto in (6, 17):
                tuples.append((proto, dst, int.from_bytes(bytes(out[hl:hl + 2]), "big"), dport))
        elif proto == 47:
            rec = (nat_addr, 0x1111, 1)           # a record on a protocol the reference's NAT refuses
        add(d, rec, out, r, V_ACCEPT if r == 0 else V_UNTOUCHED)

    for k in range(500):
        if tuples and k % 4 != 3:
            proto, remote, nport, rport = tuples[int(rng.integers(len(tuples)))]
        else:
            proto, remote, nport, rport = [6, 17][k % 2], bytes([203, 0, 113, 9]), int(rng.integers(1024, 65536)), 80
        tl = int(rng.integers(20 if proto == 6 else 8, 700))
        l4 = ["valid", "bad", "zero"][int(rng.integers(3))] if proto == 17 else ["valid", "bad"][int(rng.integers(2))]
        d = datagram(rng, proto, tl, remote, NAT_ADDR, rport, nport, opts=int(rng.integers(2)), l4=l4)
        out = d.copy()
        r = R.rr_nat(2, out.ctypes.data, out.size, nat_addr)
        rec = (0, 0, 0)
        if r == 0:
            hl = 20 + 4 * ((out[0] & 0x0F) - 5)
            rec = (int.from_bytes(bytes(out[16:20]), "little"), int.from_bytes(bytes(out[hl + 2:hl + 4]), "little"), 2)
        add(d, rec, out, r, V_ACCEPT if r == 0 else V_UNTOUCHED)

    # not handed to NAT by the stack: fragments, infeasible lengths, short transports with a record
    for k in range(60):
        proto = [6, 17][k % 2]
        d = datagram(rng, proto, 200, bytes([10, 0, 0, 5]), bytes([203, 0, 113, 7]), 4000 + k, 80,
                     frag=[0x2000, 0x2000 | 185, 370][k % 3])
        add(d, (nat_addr, 0x1234, 1), d.copy(), -9, V_FRAG)
    for k in range(30):
        d = datagram(rng, 6, 100, bytes([10, 0, 0, 6]), bytes([203, 0, 113, 7]), 5000 + k, 80)
        tot = 120 + 40 + k                        # total length past the buffer
        d[2], d[3] = tot >> 8, tot & 0xFF
        add(d, (nat_addr, 0x1234, 1), d.copy(), -9, V_MALFORMED)
    for k in range(20):
        proto = [6, 17][k % 2]
        d = datagram(rng, proto, 4 + k % 4, bytes([10, 0, 0, 7]), bytes([203, 0, 113, 7]), 6000 + k, 80)
        add(d, (nat_addr, 0x4321, 1 + k % 2), d.copy(), -9, V_MALFORMED)

    n = len(frames)
    off = np.zeros(n, np.uint64)
    avail = np.array([f.size for f in frames], np.uint32)
    pos = 0
    for i, f in enumerate(frames):
        pos += 14 + int(rng.integers(0, 3))       # Ethernet gap, odd placements too
        off[i] = pos
        pos += f.size
    buf = np.zeros(pos + 16, np.uint8)
    want = np.zeros(pos + 16, np.uint8)
    for i in range(n):
        buf[int(off[i]):int(off[i]) + frames[i].size] = frames[i]
        want[int(off[i]):int(off[i]) + frames[i].size] = wants[i]
    nat = np.zeros(n, O.NAT_DTYPE)
    nat["addr"] = [r[0] for r in recs]
    nat["port"] = [r[1] for r in recs]
    nat["dir"] = [r[2] for r in recs]
    ret = np.array(rets, np.int32)
    verdict = np.array(verdicts, np.uint8)

    # the restatement agrees with the reference on every case before anything is written
    got = buf.copy()
    desc = np.zeros(n, O.DESC_DTYPE)
    desc["off"], desc["len"] = off, avail
    on, ol, v = O.batch_ipv4_nat(got, desc, nat)
    assert np.array_equal(got, want), "oracle_batch_ipv4_nat disagrees with the reference's bytes"
    assert np.array_equal(v, verdict), np.flatnonzero(v != verdict)[:10]
    np.savez_compressed(os.path.join(OUT, "ref_nat_cases.npz"), buf=buf, off=off, avail=avail, nat=nat.view(np.uint8),
                        want=want, ret=ret, verdict=verdict)
    print(f"ref_nat_cases.npz: {n} datagrams, {int((ret == 0).sum())} translated by the reference, "
          f"{int((ret == -1).sum())} returned -1, {int((ret == -9).sum())} not handed to NAT; "
          f"{len(tuples)} outbound tuples; oracle agrees on every byte")


if __name__ == "__main__":
    main()
