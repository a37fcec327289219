#!/usr/bin/env python3
"""Golden Ethernet-burst verdicts from the reference's own compiled Ethernet + IP receive path.

Run here (where /root/reference exists):
    make -C oracle all refrx && python tests/golden/make_ref_eth.py

oracle/_ref/libref_rx.so (see make_ref_rx.py) also exports rr_eth_rx: one frame through the
reference's pico_ethernet_receive (modules/pico_ethernet.c:213-235, reached through
oracle/ref_rx_wrap.c unit 5) on an Ethernet device with the burst's MAC -- the destination filter
(own MAC, 01:00:5e, 33:33, broadcast), then pico_eth_receive's ethertype dispatch (:180-202) with
the IP version checks of pico_ipv4_ethernet_receive / pico_ipv6_ethernet_receive (:143-176) --
observed as the queue the frame lands in (IPv4, IPv6), the ARP hand-off (pico_arp_receive,
wrapped), or a discard.  Frames handed to IPv4 / IPv6 then get the reference's IP + transport
verdict on their datagram (rr_ipv4_rx / rr_ipv6_rx, as make_ref_rx.py).

Frames (seeded): the IPv4 and IPv6 datagram generators of make_ref_rx.py, ARP, LLDP and unknown
ethertypes, IP versions that do not match the ethertype; destinations: the device's MAC,
broadcast, 01:00:5e:xx, 33:33:xx, other unicast, other multicast (01:80:c2:...).  Each frame at a
random alignment in one buffer, descriptors at the Ethernet header.

Expected values: the oracle's batch_eth (oracle/pico_csum_oracle.c), asserted equal to the
reference's L2 decision for every frame and to its IP verdict wherever make_ref_rx.py's rules pin
it (`pinned`).

Output (data only): ref_eth_cases.npz -- buf, off, avail, mac, verdict, net, l4, pinned, l2 (the
reference's decision: 0 discard, 1 IPv4, 2 IPv6, 3 ARP)
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle import oracle as O  # noqa: E402
import make_ref_rx as RX  # noqa: E402

MAC = bytes.fromhex("02005e0a0b0c")
V_ACCEPT, V_NET_BAD, V_L4_BAD, V_MALFORMED, V_FRAG, V_DROP_L2, V_ARP, V_IPV6 = 1, 2, 4, 8, 16, 32, 64, 128


def gen_frames(rng, n):
    v4 = RX.gen_v4(rng, n)
    v6 = RX.gen_v6(rng, n)
    out = []
    for i in range(n):
        k = rng.random()
        if k < 0.42:
            body, et = v4[i][0], 0x0800
        elif k < 0.80:
            body, et = v6[i][0], 0x86DD
        elif k < 0.86:
            body, et = rng.integers(0, 256, 28).astype(np.uint8).tobytes(), 0x0806
        elif k < 0.90:
            body, et = rng.integers(0, 256, int(rng.integers(46, 200))).astype(np.uint8).tobytes(), \
                int(rng.choice([0x88CC, 0x1234, 0x8100, 0x0000]))
        elif k < 0.95:
            body, et = v6[i][0], 0x0800                    # IPv6 behind the IPv4 ethertype
        else:
            body, et = v4[i][0], 0x86DD                    # and the other way round
        k = rng.random()
        if k < 0.6:
            dst = MAC
        elif k < 0.7:
            dst = b"\xff" * 6
        elif k < 0.78:
            dst = bytes([1, 0, 0x5E]) + rng.integers(0, 256, 3).astype(np.uint8).tobytes()
        elif k < 0.86:
            dst = bytes([0x33, 0x33]) + rng.integers(0, 256, 4).astype(np.uint8).tobytes()
        elif k < 0.94:
            dst = bytes([0x02, 0x11]) + rng.integers(0, 256, 4).astype(np.uint8).tobytes()
        else:
            dst = bytes([1, 0x80, 0xC2, 0, 0, int(rng.integers(0, 16))])
        src = bytes([0x02]) + rng.integers(0, 256, 5).astype(np.uint8).tobytes()
        fr = dst + src + bytes([et >> 8, et & 0xFF]) + body
        out.append((fr, len(fr)))
    return out


def main() -> None:
    if not os.path.exists(RX.REF_RX):
        sys.exit(f"{RX.REF_RX} missing: run `make -C oracle refrx` first")
    R = RX.ref_lib()
    R.rr_eth_init.argtypes = [ctypes.c_char_p]
    R.rr_eth_rx.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    assert R.rr_eth_init(MAC) == 0
    rng = np.random.default_rng(20261019)
    frames = gen_frames(rng, 6000)
    buf, off, av = RX.pack(frames, rng)
    desc = np.zeros(len(frames), O.DESC_DTYPE)
    desc["off"], desc["len"] = off, av
    on, ol, ov = O.batch_eth(buf, desc, mac=MAC)
    pinned = np.zeros(len(frames), bool)
    l2 = np.zeros(len(frames), np.uint8)
    for i, (fr, a) in enumerate(frames):
        x = np.frombuffer(fr, np.uint8).copy()
        r = R.rr_eth_rx(x.ctypes.data, a)
        assert r >= 0
        l2[i] = r
        v = int(ov[i])
        if r == 0:
            assert v == V_DROP_L2, (i, v, fr[:20].hex())
            pinned[i] = True
            continue
        if r == 3:
            assert v == V_ARP, (i, v)
            pinned[i] = True
            continue
        d, da = x[14:], a - 14
        if r == 1:
            assert not (v & V_IPV6) and v in (V_ACCEPT, V_NET_BAD, V_L4_BAD, V_MALFORMED, V_FRAG), (i, v)
            if da < 20 or RX.v4_reads_past(bytes(d), da):
                continue
            rr = R.rr_ipv4_rx(np.ascontiguousarray(d).ctypes.data, da)
            if rr & 1:
                want = V_FRAG
            elif rr & 2:
                want = V_ACCEPT if (((rr >> 8) & 0xFF) not in (6, 17) or rr & 4) else V_L4_BAD
            else:
                ihl = int(d[0]) & 0x0F
                nl = 20 + (4 * (ihl - 5) if ihl > 5 else 0)
                lengths_ok = ((((int(d[2]) << 8) | int(d[3])) - nl) & 0xFFFF) <= ((da - 20) & 0xFFFF)
                want = V_NET_BAD if (not (rr & 16) and lengths_ok) else V_MALFORMED
            assert v == want, (i, v, want, bytes(d).hex())
            pinned[i] = True
        else:
            assert v & V_IPV6, (i, v)
            v &= ~V_IPV6
            if da < 40:
                continue
            k, nl, pr = O.ipv6_walk(d[:da])
            if k == O.WALK_BAD:
                continue
            rn, rp = ctypes.c_uint32(0), ctypes.c_uint32(0)
            rr = R.rr_ipv6_rx(np.ascontiguousarray(d).ctypes.data, da, ctypes.byref(rn), ctypes.byref(rp))
            assert (rr & 3) == k, (i, rr, k)
            if k == O.WALK_DROP:
                assert v == V_MALFORMED
                pinned[i] = True
            elif k == O.WALK_FRAG:
                assert v == V_FRAG
                pinned[i] = True
            else:
                plen = (int(d[4]) << 8) | int(d[5])
                tl = (plen - (nl - 40)) & 0xFFFF
                if nl + tl > da or (pr == 17 or d[9] == 17) and nl + 8 > da:
                    continue
                if pr in (6, 17):
                    assert v == (V_ACCEPT if rr & 4 else V_L4_BAD), (i, rr, v)
                    pinned[i] = True
    np.savez_compressed(os.path.join(HERE, "ref_eth_cases.npz"), buf=buf, off=off, avail=av,
                        mac=np.frombuffer(MAC, np.uint8), verdict=ov, net=on, l4=ol, pinned=pinned, l2=l2)
    print("frames", len(frames), "pinned", int(pinned.sum()), "l2", dict(zip(*[x.tolist() for x in np.unique(l2, return_counts=True)])),
          "verdicts", dict(zip(*[x.tolist() for x in np.unique(ov, return_counts=True)])))


if __name__ == "__main__":
    main()
