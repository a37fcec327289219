#!/usr/bin/env python3
"""Golden RX verdicts from the reference's own compiled RX path.

Run here (where /root/reference exists):
    make -C oracle all refrx && python tests/golden/make_ref_rx.py

oracle/_ref/libref_rx.so is the whole reference stack compiled from /root/reference with
modules/pico_ipv4.c, modules/pico_ipv6.c and stack/pico_socket.c reached through
oracle/ref_rx_wrap.c (their static RX functions exported, nothing modified) and driven by
oracle/ref_rx_driver.c, which observes the hand-offs with linker --wrap:
  IPv4: pico_ipv4_process_in (modules/pico_ipv4.c:381-470) -- lengths, pico_ipv4_crc_check,
        pico_ipv4_is_valid_src, the evil bit, IHL < 5, the fragment hand-off to
        pico_ipv4_process_frag, delivery -- then pico_transport_crc_check
        (stack/pico_socket.c:1916-1968) on what it delivers
  IPv6: pico_ipv6_extension_headers (modules/pico_ipv6.c:659-809, with the sequence check,
        hop-by-hop / routing / fragment / destination-option processing) and, for TCP / UDP,
        pico_transport_crc_check with the byte-9 dispatch the reference really performs.

Datagrams (seeded; two families):
  v4: IHL 0-15 (options), TCP / UDP / ICMPv4 / GRE, valid or corrupted header and transport
      checksums, DF / MF / offsets / the evil bit, broadcast / multicast / loopback sources,
      truncated buffers, infeasible total lengths
  v6: random extension-header chains (hop-by-hop with Pad1 / PadN / router alert / unknown
      options of every action, routing with segments left of type 0 / 2 / 4, fragment headers
      with M and offsets, destination options, ESP, no next header, invalid next headers),
      TCP / UDP / ICMPv6 with valid or corrupted checksums, any byte 9, payload lengths that
      are or are not a multiple of 8, truncated buffers
Each datagram is placed at a random alignment in one buffer.

Expected verdict (include/pico_csum.h): v4 from the reference run (pinned); v6 the walk outcome
and, for TCP / UDP, the transport check from the reference run (pinned); ICMPv6 types and the
read-past-the-frame bounds of the batch API come from oracle/pico_csum_oracle.c (the checksum
VALUES of every transport are the oracle's, themselves pinned by ref_callers.npz).  Datagrams on
which the reference would read past its buffer or never terminate cannot be run on it: their
expectation is the oracle's (MALFORMED) and `pinned` is False for them.

Output (data only): ref_rx_cases.npz
  v4_buf, v4_off, v4_avail, v4_verdict, v4_net, v4_l4, v4_pinned
  v6_buf, v6_off, v6_avail, v6_verdict, v6_l4, v6_pinned, v6_net_len (walk result, 0 if none)
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

OUT = HERE
REF_RX = os.path.join(ROOT, "oracle", "_ref", "libref_rx.so")
DSTS4 = [bytes([192, 168, 7, i]) for i in range(1, 9)]
V_ACCEPT, V_NET_BAD, V_L4_BAD, V_MALFORMED, V_FRAG = 1, 2, 4, 8, 16


def ref_lib():
    R = ctypes.CDLL(REF_RX)
    R.rr_init.restype = ctypes.c_int
    R.rr_ipv4_rx.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    R.rr_ipv4_link.argtypes = [ctypes.c_uint32]
    R.rr_ipv6_rx.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    if R.rr_init() != 0:
        raise RuntimeError("rr_init failed")
    for d in DSTS4:
        R.rr_ipv4_link(int.from_bytes(d, "little"))
    return R


def _fin(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    c = ~s & 0xFFFF
    return ((c >> 8) | (c << 8)) & 0xFFFF


def _sum(b: bytes, s: int = 0) -> int:
    return O.adder(s, np.frombuffer(bytes(b), np.uint8)) if len(b) else s


def gen_v4(rng, n):
    """Random IPv4 datagrams (see module doc); returns a list of byte strings and avails."""
    out = []
    while len(out) < n:
        ihl = int(rng.choice([5, 5, 5, 5, 6, 8, 15, 4, 3, 0]))
        hl = 20 + (4 * (ihl - 5) if ihl > 5 else 0)
        proto = int(rng.choice([6, 17, 1, 47, 6, 17, 6]))
        tl = int(rng.integers(0, 300))
        if proto == 6:
            tl = max(tl, 20)
        if proto in (17, 1):
            tl = max(tl, 8)
        h = bytearray(hl)
        h[0] = 0x40 | ihl
        tot = hl + tl
        h[2], h[3] = tot >> 8, tot & 0xFF
        h[4], h[5] = int(rng.integers(256)), int(rng.integers(256))
        k = rng.random()
        fr = 0x4000
        if k < 0.15:
            fr = 0x2000 | int(rng.integers(0, 200))          # first / middle fragments
        elif k < 0.25:
            fr = int(rng.integers(1, 0x2000))                # last fragments
        elif k < 0.30:
            fr = 0x8000 | int(rng.choice([0, 0x4000, 0x2000]))   # the evil bit
        elif k < 0.45:
            fr = 0
        h[6], h[7] = fr >> 8, fr & 0xFF
        h[8], h[9] = 64, proto
        src = bytes([10, int(rng.integers(256)), int(rng.integers(256)), int(rng.integers(1, 255))])
        k = rng.random()
        if k < 0.03:
            src = b"\xff\xff\xff\xff"
        elif k < 0.06:
            src = bytes([int(rng.integers(224, 256)), 1, 2, 3])
        elif k < 0.08:
            src = bytes([127, 0, 0, int(rng.integers(1, 255))])
        h[12:16] = src
        h[16:20] = DSTS4[int(rng.integers(0, len(DSTS4)))]
        for i in range(20, hl):
            h[i] = 1                                          # NOP options
        t = bytearray(rng.integers(0, 256, tl).astype(np.uint8).tobytes())
        if proto == 6:
            t[12], t[13], t[16], t[17] = 0x50, 0x18, 0, 0
        if proto == 17:
            t[4], t[5], t[6], t[7] = tl >> 8, tl & 0xFF, 0, 0
        if proto == 1:
            t[2], t[3] = 0, 0
        if proto in (6, 17) and rng.random() < 0.85:
            ph = bytes(h[12:20]) + bytes([0, proto, tl >> 8, tl & 0xFF])
            c = _fin(_sum(bytes(t), _sum(ph)))
            x = 16 if proto == 6 else 6
            t[x], t[x + 1] = c >> 8, c & 0xFF
            if rng.random() < 0.2:
                t[int(rng.integers(0, tl))] ^= 1 << int(rng.integers(8))
        c = _fin(_sum(bytes(h)))
        h[10], h[11] = c >> 8, c & 0xFF
        if rng.random() < 0.1:
            h[int(rng.integers(0, hl))] ^= 1 << int(rng.integers(8))
        d = bytearray(bytes(h) + bytes(t) + rng.integers(0, 256, int(rng.integers(0, 6))).astype(np.uint8).tobytes())
        if rng.random() < 0.04:
            tot2 = int(rng.integers(0, 400))
            d[2], d[3] = tot2 >> 8, tot2 & 0xFF
        avail = len(d)
        if rng.random() < 0.08:
            avail = int(rng.integers(20, len(d) + 1))
        out.append((bytes(d[:avail]), avail))
    return out


def _opts(rng, h):
    """Fill option bytes [2, len(h)) of a hop-by-hop / destination-options header."""
    p = 2
    while p < len(h):
        k = rng.random()
        room = len(h) - p
        if k < 0.3 or room < 2:
            h[p] = 0
            p += 1
        elif k < 0.6:
            ln = room - 2 if rng.random() < 0.6 else int(rng.integers(0, room - 1))
            h[p], h[p + 1] = 1, ln
            p += 2 + ln
        elif k < 0.75 and room >= 4:
            h[p], h[p + 1] = 5, int(rng.choice([2, 2, 0]))
            p += 2 + h[p + 1]
        else:
            h[p], h[p + 1] = int(rng.choice([0x3E, 0x7E, 0x9E, 0xDE, 201, 0x1F])), 0
            p += 2


def gen_v6(rng, n):
    out = []
    while len(out) < n:
        nh = int(rng.choice([0, 0, 1, 1, 2, 3, 4]))
        types = [int(rng.choice([0, 43, 44, 60, 60, 0, 44])) for _ in range(nh)]
        if types and rng.random() < 0.7 and 0 in types:
            types.remove(0)
            types.insert(0, 0)                                # hop-by-hop first, mostly
        last = int(rng.choice([6, 17, 58, 6, 17, 58, 59, 50, 51, 47]))
        seq = types + [last]
        body = bytearray()
        for i, t in enumerate(types):
            nx = seq[i + 1]
            if t == 44:
                h = bytearray(8)
                h[0] = nx
                off = int(rng.integers(0, 200)) << 3 if rng.random() < 0.6 else 0
                m = int(rng.random() < 0.6)
                om = off | m
                h[2], h[3] = om >> 8, om & 0xFF
                h[4:8] = rng.integers(0, 256, 4).astype(np.uint8).tobytes()
            else:
                L = int(rng.choice([0, 0, 0, 1, 2]))
                h = bytearray(8 * (L + 1))
                h[0], h[1] = nx, L
                if t == 43:
                    h[2], h[3] = int(rng.choice([0, 2, 4])), int(rng.choice([0, 0, 1, 3]))
                else:
                    _opts(rng, h)
            body += h
        proto = last
        tl = int(rng.integers(0, 240))
        if proto == 6:
            tl = max(tl, 20)
        if proto == 17:
            tl = max(tl, 8)
        if proto == 58:
            tl = max(tl, 4)
        if rng.random() < 0.5:
            tl = (tl + 7) & ~7                               # payload multiple of 8, often
        t = bytearray(rng.integers(0, 256, tl).astype(np.uint8).tobytes())
        hdr = bytearray(40)
        hdr[0] = 0x60
        hdr[6] = seq[0]
        hdr[7] = 64
        hdr[8:40] = rng.integers(0, 256, 32).astype(np.uint8).tobytes()
        if rng.random() < 0.3:
            hdr[9] = int(rng.choice([6, 17]))                 # the byte pico_transport_crc_check reads
        plen = len(body) + tl
        if proto == 17:
            t[4], t[5], t[6], t[7] = plen >> 8 & 0xFF, plen & 0xFF, 0, 0
        if proto == 58:
            t[0] = int(rng.choice([128, 129, 133, 134, 135, 136, 130, 143, 1]))
            t[2], t[3] = 0, 0
        if proto == 6:
            t[16], t[17] = 0, 0
        if proto in (6, 17, 58) and rng.random() < 0.85:
            pn = proto if proto == 58 or rng.random() < 0.7 else int(hdr[9])
            ph = bytes(hdr[8:40]) + tl.to_bytes(4, "big") + bytes([0, 0, 0, pn])
            c = _fin(_sum(bytes(t), _sum(ph)))
            x = {6: 16, 17: 6, 58: 2}[proto]
            t[x], t[x + 1] = c >> 8, c & 0xFF
            if rng.random() < 0.2:
                t[int(rng.integers(0, tl))] ^= 1 << int(rng.integers(8))
        if rng.random() < 0.15:
            plen = int(rng.integers(0, plen + 24))
        hdr[4], hdr[5] = plen >> 8 & 0xFF, plen & 0xFF
        d = bytes(hdr) + bytes(body) + bytes(t) + rng.integers(0, 256, int(rng.integers(0, 6))).astype(np.uint8).tobytes()
        avail = len(d)
        if rng.random() < 0.08:
            avail = int(rng.integers(40, len(d) + 1))
        out.append((d[:avail], avail))
    return out


def pack(items, rng):
    """Datagrams into one buffer at random alignments: (buf, off, avail)."""
    offs, pos = [], 0
    for d, _ in items:
        pos += int(rng.integers(0, 16))
        offs.append(pos)
        pos += len(d)
    buf = np.zeros(pos + 16, np.uint8)
    for (d, _), o in zip(items, offs):
        buf[o:o + len(d)] = np.frombuffer(d, np.uint8)
    return buf, np.array(offs, np.uint64), np.array([a for _, a in items], np.uint32)


def v4_reads_past(d: bytes, avail: int) -> bool:
    """Would the reference read past the buffer (the oracle's MALFORMED bounds)?"""
    ihl = d[0] & 0x0F
    nl = 20 + (4 * (ihl - 5) if ihl > 5 else 0)
    tot = (d[2] << 8) | d[3]
    tl = (tot - nl) & 0xFFFF
    mx = (avail - 20) & 0xFFFF
    return nl > avail or (tl <= mx and nl + tl > avail) or (d[9] == 17 and nl + 8 > avail)


def main() -> None:
    if not os.path.exists(REF_RX):
        sys.exit(f"{REF_RX} missing: run `make -C oracle refrx` first")
    R = ref_lib()
    rng = np.random.default_rng(20261017)
    # ---- IPv4
    v4 = gen_v4(rng, 5000)
    buf4, off4, av4 = pack(v4, rng)
    desc = np.zeros(len(v4), O.DESC_DTYPE)
    desc["off"], desc["len"] = off4, av4
    on, ol, ov = O.batch_ipv4(buf4, desc)
    pin4 = np.zeros(len(v4), bool)
    for i, (d, a) in enumerate(v4):
        if v4_reads_past(d, a):
            continue
        x = np.frombuffer(d, np.uint8).copy()
        r = R.rr_ipv4_rx(x.ctypes.data, a)
        if r & 1:
            rv = V_FRAG
        elif r & 2:
            rv = V_ACCEPT if (((r >> 8) & 0xFF) not in (6, 17) or r & 4) else V_L4_BAD
        else:
            ihl = d[0] & 0x0F
            nl = 20 + (4 * (ihl - 5) if ihl > 5 else 0)
            lengths_ok = ((((d[2] << 8) | d[3]) - nl) & 0xFFFF) <= ((a - 20) & 0xFFFF)
            rv = V_NET_BAD if (not (r & 16) and lengths_ok) else V_MALFORMED
        assert rv == ov[i], (i, rv, int(ov[i]), d.hex())
        pin4[i] = True
    # ---- IPv6
    v6 = gen_v6(rng, 5000)
    buf6, off6, av6 = pack(v6, rng)
    desc = np.zeros(len(v6), O.DESC_DTYPE)
    desc["off"], desc["len"] = off6, av6
    l6, vv6 = O.batch_ipv6(buf6, desc)
    pin6 = np.zeros(len(v6), bool)
    nl6 = np.zeros(len(v6), np.uint32)
    for i, (d, a) in enumerate(v6):
        x = np.frombuffer(d, np.uint8).copy()
        k, nl, pr = O.ipv6_walk(x)
        if k == O.WALK_BAD:
            continue
        rn, rp = ctypes.c_uint32(0), ctypes.c_uint32(0)
        r = R.rr_ipv6_rx(x.ctypes.data, a, ctypes.byref(rn), ctypes.byref(rp))
        assert (r & 3) == k and (k != 1 or (rn.value, rp.value) == (nl, pr)), (i, r, k, nl, pr, d.hex())
        if k == O.WALK_DROP:
            assert vv6[i] == V_MALFORMED
            pin6[i] = True
        elif k == O.WALK_FRAG:
            assert vv6[i] == V_FRAG
            pin6[i] = True
        else:
            nl6[i] = nl
            plen = (d[4] << 8) | d[5]
            tl = (plen - (nl - 40)) & 0xFFFF
            if nl + tl > a or (pr == 17 or d[9] == 17) and nl + 8 > a:
                continue                                      # the batch API's bounds: oracle only
            if pr in (6, 17):
                want = V_ACCEPT if (r & 4) else V_L4_BAD
                assert vv6[i] == want, (i, r, int(vv6[i]), d.hex())
                pin6[i] = True
    np.savez_compressed(os.path.join(OUT, "ref_rx_cases.npz"),
                        v4_buf=buf4, v4_off=off4, v4_avail=av4, v4_verdict=ov, v4_net=on, v4_l4=ol, v4_pinned=pin4,
                        v6_buf=buf6, v6_off=off6, v6_avail=av6, v6_verdict=vv6, v6_l4=l6, v6_pinned=pin6,
                        v6_net_len=nl6)
    print("v4:", len(v4), "pinned", int(pin4.sum()), "verdicts", dict(zip(*[x.tolist() for x in np.unique(ov, return_counts=True)])))
    print("v6:", len(v6), "pinned", int(pin6.sum()), "verdicts", dict(zip(*[x.tolist() for x in np.unique(vv6, return_counts=True)])))


if __name__ == "__main__":
    main()
