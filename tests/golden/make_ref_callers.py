#!/usr/bin/env python3
"""Golden transport checksums from the reference's own compiled CALLERS.

Run here (where /root/reference exists):
    make -C oracle refcallers && python tests/golden/make_ref_callers.py

oracle/_ref/libref_callers.so is the reference's modules/pico_tcp.c, pico_udp.c,
pico_icmp6.c, pico_mld.c and stack/pico_frame.c, compiled unmodified, behind
oracle/ref_callers_shim.c (which allocates each struct pico_frame with the
reference's pico_frame_alloc and calls):
  pico_tcp_checksum_ipv4  modules/pico_tcp.c:422-446   RX (f->sock NULL) and TX (socket addresses)
  pico_udp_checksum_ipv4  modules/pico_udp.c:36-60     RX (stored crc != 0, pico_socket.c:1941)
  pico_tcp_checksum_ipv6  modules/pico_tcp.c:449-475   RX and TX
  pico_udp_checksum_ipv6  modules/pico_udp.c:63-92     RX (crc != 0) and TX
  pico_icmp6_checksum     modules/pico_icmp6.c:38-55   RX and TX (crc zeroed first)
  pico_mld_checksum       modules/pico_mld.c:421-437   MLDv2 reports behind an 8-byte router alert
over the datagrams of ipv4_cases.npz / ipv6_cases.npz (same bytes, same offsets), for
every datagram the IP layer hands to the transport.  f->net_len / f->transport_len
are set as pico_ipv4_process_in (pico_ipv4.c:392-405) and pico_ipv6_process_in
(pico_ipv6.c:707-800, the descriptor seed for extension headers) derive them.

This pins the fused kernels' transport checksums to the reference's own caller code
(VERDICT r01 "next" item 2) rather than to the Python restatement in make_golden.py:
the script asserts the two agree, and tests compare the GPU kernels with these arrays.

Output (data only): ref_callers.npz
  v4_rx / v4_tx  int32[n4]  reference value, -1 where the stack makes no such call
  v6_rx / v6_tx  int32[n6]  same for the IPv6 datagrams
  mld_buf, mld_net, mld_size, mld_rx, mld_tx: MLDv2 report datagrams (IPv6 header, hop-by-hop
                 router alert, report) and pico_mld_checksum over them as they are (rx) and with
                 the report's crc zeroed (tx)
and eth_cases.npz: a mixed Ethernet burst (IPv4 / IPv6 / ARP / other ethertypes, MAC filter
cases) with the oracle_batch_eth expectations (pico_ethernet.c:180-235 dispatch restated in
oracle/pico_csum_oracle.c), every transport value of an IP frame checked against the
reference callers above.  The dispatch itself is static in pico_ethernet.c and needs the
device layer, so that part is restated, not compiled ("parity unpinned" for the dispatch).
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
from picotcp_amd import synth  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(ROOT, "oracle", "_ref", "libref_callers.so")
RC_TCP4, RC_UDP4, RC_TCP6, RC_UDP6, RC_ICMP6, RC_MLD = range(6)
MAL, NET_BAD, FRAG = 8, 2, 16
NO_L4 = (MAL, NET_BAD, FRAG)          # verdicts where the stack makes no transport call


def load():
    lib = ctypes.CDLL(LIB)
    lib.rc_checksum.restype = ctypes.c_int
    lib.rc_checksum.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_int]
    return lib


def call(lib, which, buf: np.ndarray, off: int, size: int, net_len: int, tl: int, tx: bool) -> int:
    d = np.ascontiguousarray(buf[off:off + size])
    r = lib.rc_checksum(which, d.ctypes.data, size, net_len, tl, 1 if tx else 0)
    assert r >= 0, (which, off, size, net_len, tl, tx)
    return r


def ipv4(lib, cases) -> tuple[np.ndarray, np.ndarray]:
    n = cases["net"].size
    rx = np.full(n, -1, dtype=np.int32)
    tx = np.full(n, -1, dtype=np.int32)
    for i in range(n):
        o, a = int(cases["net"][i]), int(cases["avail"][i])
        for is_tx, buf, out, verdict in ((False, cases["buf"], rx, cases["rx_verdict"]),
                                         (True, cases["tx_buf"], tx, cases["tx_verdict"])):
            if verdict[i] in NO_L4 or a < 20:
                continue                                  # the IP layer discards it / hands it to reassembly
            h = buf[o:o + a]
            ihl = int(h[0]) & 0xF
            hl = 20 + (4 * (ihl - 5) if ihl > 5 else 0)
            tl = ((int(h[2]) << 8 | int(h[3])) - hl) & 0xFFFF          # pico_ipv4.c:395
            proto = int(h[9])
            if not is_tx:
                if proto == 6:
                    out[i] = call(lib, RC_TCP4, buf, o, a, hl, tl, False)
                elif proto == 17 and (h[hl + 6] or h[hl + 7]):         # pico_socket.c:1941
                    out[i] = call(lib, RC_UDP4, buf, o, a, hl, tl, False)
            elif proto == 6 and tl >= 20:
                out[i] = call(lib, RC_TCP4, buf, o, a, hl, tl, True)
    return rx, tx


def ipv6(lib, cases, nxthdr_dispatch: bool = False) -> tuple[np.ndarray, np.ndarray]:
    """RX: TCP / UDP checked as pico_transport_crc_check dispatches them -- on byte 9 of the
    header (stack/pico_socket.c:1919-1923) -- or, with nxthdr_dispatch, by the transport's own
    protocol; ICMPv6 by pico_icmp6_checksum."""
    n = cases["net"].size
    rx = np.full(n, -1, dtype=np.int32)
    tx = np.full(n, -1, dtype=np.int32)
    which = {6: RC_TCP6, 17: RC_UDP6, 58: RC_ICMP6}
    need = {6: 20, 17: 8, 58: 4}
    rxv = cases["rx_verdict_nx"] if nxthdr_dispatch else cases["rx_verdict"]
    for i in range(n):
        o, a, seed = int(cases["net"][i]), int(cases["avail"][i]), int(cases["seed"][i])
        for is_tx, buf, out, verdict in ((False, cases["buf"], rx, rxv),
                                         (True, cases["tx_buf"], tx, cases["tx_verdict"])):
            if verdict[i] in NO_L4 or a < 40:
                continue
            h = buf[o:o + a]
            net_len, proto = (seed & 0xFFFF, (seed >> 16) & 0xFF) if seed else (40, int(h[6]))
            tl = ((int(h[4]) << 8 | int(h[5])) - (net_len - 40)) & 0xFFFF   # pico_ipv6.c:790
            if proto not in which:
                continue
            if not is_tx:
                if proto in (6, 17) and not nxthdr_dispatch:
                    proto = int(h[9])                      # net_hdr->proto through the IPv4 cast
                    if proto not in (6, 17):
                        continue
                if proto == 17 and not (h[net_len + 6] or h[net_len + 7]):
                    continue
                out[i] = call(lib, which[proto], buf, o, a, net_len, tl, False)
            elif tl >= need[proto]:
                out[i] = call(lib, which[proto], buf, o, a, net_len, tl, True)
    return rx, tx


def mld(lib, n: int = 96):
    """MLDv2 reports as pico_mld sends them: IPv6 header (next header 0), an 8-byte
    hop-by-hop router alert (MLD_ROUTER_ALERT_LEN, pico_mld.c:38), the report
    (type 143) with random records; transport = router alert + report."""
    rng = np.random.default_rng(7373)
    rep = rng.integers(8, 400, n).astype(np.uint32)           # report bytes
    tl = rep + 8
    lens = 40 + tl
    starts = np.zeros(n, dtype=np.uint64)
    starts[1:] = np.cumsum(lens.astype(np.uint64) + 2)[:-1]   # 2-byte gaps: odd / even offsets vary
    starts += np.uint64(1)
    buf = synth.random_bytes(0x313D, int(starts[-1]) + int(lens[-1]) + 8)
    rx = np.zeros(n, dtype=np.int32)
    tx = np.zeros(n, dtype=np.int32)
    for i in range(n):
        o = int(starts[i])
        buf[o] = 0x60
        buf[o + 4] = tl[i] >> 8
        buf[o + 5] = tl[i] & 0xFF
        buf[o + 6] = 0                                         # hop-by-hop
        buf[o + 7] = 1
        buf[o + 40:o + 48] = [58, 0, 5, 2, 0, 0, 1, 0]         # router alert (RFC 2711)
        buf[o + 48] = 143
        buf[o + 49] = 0
        rx[i] = call(lib, RC_MLD, buf, o, int(lens[i]), 40, int(tl[i]), False)
        tx[i] = call(lib, RC_MLD, buf, o, int(lens[i]), 40, int(tl[i]), True)
    return dict(mld_buf=buf, mld_net=starts, mld_size=lens, mld_rx=rx, mld_tx=tx)


MAC = bytes.fromhex("02005e0a0b0c")


def eth(lib, n: int = 1536):
    """The Ethernet front end (oracle_batch_eth: pico_ethernet.c:180-235 dispatch, then the
    IPv4 / IPv6 logic) over a mixed burst (synth.eth_batch): TX expectations on the
    zero-crc frames; the checksums then stored as the reference TX path does (UDP over IPv4
    with a real checksum so that RX verifies it); seeded corruptions; RX expectations with
    and without the destination-MAC filter.  Every transport value of an IP frame is also
    checked against the reference's own callers."""
    from oracle import oracle as O
    buf, off, flen, seeds, kind = synth.eth_batch(n, seed=31, mac=MAC)
    desc = np.zeros(n, dtype=[("off", "<u8"), ("len", "<u4"), ("seed", "<u4")])
    desc["off"], desc["len"], desc["seed"] = off, flen, seeds
    tx_buf = buf.copy()
    tn, tl4, tv = O.batch_eth(tx_buf, desc, tx=True)
    rx_buf = tx_buf.copy()
    checked = 0
    for i in range(n):
        o = int(off[i]) + 14
        if tv[i] == 16:                                       # IPv4 fragment: its header checksum only
            rx_buf[o + 10], rx_buf[o + 11] = tn[i] >> 8, tn[i] & 0xFF
        if tv[i] == 1:                                        # IPv4, accepted
            ihl = int(rx_buf[o]) & 0xF
            hl = 20 + (4 * (ihl - 5) if ihl > 5 else 0)
            tlen = ((int(rx_buf[o + 2]) << 8) | int(rx_buf[o + 3])) - hl
            proto = int(rx_buf[o + 9])
            rx_buf[o + 10], rx_buf[o + 11] = tn[i] >> 8, tn[i] & 0xFF
            if proto in (6, 1):
                x = o + hl + (16 if proto == 6 else 2)
                rx_buf[x], rx_buf[x + 1] = tl4[i] >> 8, tl4[i] & 0xFF
                if proto == 6:
                    assert call(lib, RC_TCP4, tx_buf, o, int(flen[i]) - 14, hl, tlen, True) == tl4[i]
                    checked += 1
            elif proto == 17:
                c = call(lib, RC_UDP4, rx_buf, o, int(flen[i]) - 14, hl, tlen, True)
                rx_buf[o + hl + 6], rx_buf[o + hl + 7] = c >> 8, c & 0xFF
        elif tv[i] == (1 | 128):                              # IPv6, accepted
            sd = int(seeds[i])
            net_len, proto = (sd & 0xFFFF, sd >> 16) if sd else (40, int(rx_buf[o + 6]))
            tlen = ((int(rx_buf[o + 4]) << 8) | int(rx_buf[o + 5])) - (net_len - 40)
            xo = {6: 16, 17: 6, 58: 2}.get(proto)
            if xo is not None:
                which = {6: RC_TCP6, 17: RC_UDP6, 58: RC_ICMP6}[proto]
                assert call(lib, which, tx_buf, o, int(flen[i]) - 14, net_len, tlen, True) == tl4[i]
                checked += 1
                rx_buf[o + net_len + xo], rx_buf[o + net_len + xo + 1] = tl4[i] >> 8, tl4[i] & 0xFF
    rng = np.random.default_rng(3131)
    for i in range(n):                                        # corruptions (index-stable)
        r = rng.random()
        o, fl = int(off[i]), int(flen[i])
        if r < 0.7:
            continue
        if r < 0.8:
            rx_buf[o + 14 + int(rng.integers(0, max(1, fl - 14)))] ^= 0x10          # header / payload bit
        elif r < 0.85:
            desc["len"][i] = int(rng.integers(0, 40))                               # truncated frame
        elif r < 0.9:
            rx_buf[o + 12], rx_buf[o + 13] = 0x81, 0x00                            # VLAN tag: not handled
        else:
            rx_buf[o:o + 6] = np.frombuffer(bytes([0x02, 0x99, 0x88, 0x77, 0x66, 0x55]), np.uint8)
    rn, rl4, rv = O.batch_eth(rx_buf, desc, mac=MAC)
    rn_nomac, rl4_nomac, rv_nomac = O.batch_eth(rx_buf, desc)
    rn_nx, rl4_nx, rv_nx = O.batch_eth(rx_buf, desc, mac=MAC, nxthdr_dispatch=True)
    for i in range(n):                                        # RX transport values vs the callers
        o, a = int(off[i]) + 14, int(desc["len"][i]) - 14
        if (rv[i] & 0x7F) in NO_L4 or a <= 0 or rl4[i] == 0 and not (rv[i] & 4):
            continue
        if rv[i] & 128:
            sd = int(seeds[i])
            if sd:
                net_len, proto = sd & 0xFFFF, sd >> 16
            else:                                             # the extension-header walk (pinned separately)
                k, net_len, proto = O.ipv6_walk(rx_buf[o:o + a])
                if k != O.WALK_PROTO:
                    continue
            tlen = (((int(rx_buf[o + 4]) << 8) | int(rx_buf[o + 5])) - (net_len - 40)) & 0xFFFF
            if proto in (6, 17):
                proto = int(rx_buf[o + 9])                    # pico_transport_crc_check's byte-9 dispatch
            which = {6: RC_TCP6, 17: RC_UDP6, 58: RC_ICMP6}.get(proto)
            if which is not None:
                assert call(lib, which, rx_buf, o, a, net_len, tlen, False) == rl4[i], i
                checked += 1
        elif rv[i] & 7:
            ihl = int(rx_buf[o]) & 0xF
            hl = 20 + (4 * (ihl - 5) if ihl > 5 else 0)
            tlen = (((int(rx_buf[o + 2]) << 8) | int(rx_buf[o + 3])) - hl) & 0xFFFF
            proto = int(rx_buf[o + 9])
            if proto in (6, 17):
                assert call(lib, RC_TCP4 if proto == 6 else RC_UDP4, rx_buf, o, a, hl, tlen, False) == rl4[i], i
                checked += 1
    print(f"eth: {n} frames, {checked} transport values checked against the reference callers;",
          "RX verdicts", dict(zip(*[x.tolist() for x in np.unique(rv, return_counts=True)])))
    return dict(tx_buf=tx_buf, buf=rx_buf, off=off, flen=flen, rx_len=desc["len"].copy(), seed=seeds, kind=kind,
                mac=np.frombuffer(MAC, np.uint8).copy(), tx_net=tn, tx_l4=tl4, tx_verdict=tv,
                rx_net=rn, rx_l4=rl4, rx_verdict=rv, rx_net_nomac=rn_nomac, rx_l4_nomac=rl4_nomac,
                rx_verdict_nomac=rv_nomac, rx_l4_nx=rl4_nx, rx_verdict_nx=rv_nx)


def main() -> None:
    if not os.path.exists(LIB):
        sys.exit(f"{LIB} missing: run `make -C oracle refcallers` first")
    lib = load()
    c4 = dict(np.load(os.path.join(OUT, "ipv4_cases.npz")))
    c6 = dict(np.load(os.path.join(OUT, "ipv6_cases.npz")))
    v4_rx, v4_tx = ipv4(lib, c4)
    v6_rx, v6_tx = ipv6(lib, c6)
    v6_rx_nx, _ = ipv6(lib, c6, nxthdr_dispatch=True)
    # the Python restatement behind ipv4_cases / ipv6_cases must agree with the reference callers
    for name, got, exp in (("v4_rx", v4_rx, c4["rx_l4"]), ("v4_tx", v4_tx, c4["tx_l4"]),
                           ("v6_rx", v6_rx, c6["rx_l4"]), ("v6_tx", v6_tx, c6["tx_l4"]),
                           ("v6_rx_nx", v6_rx_nx, c6["rx_l4_nx"])):
        m = got >= 0
        bad = np.flatnonzero(got[m] != exp[m].astype(np.int32))
        assert bad.size == 0, (name, bad[:10])
        print(f"{name}: {int(m.sum())} reference caller values, all equal to the restatement")
    out = dict(v4_rx=v4_rx, v4_tx=v4_tx, v6_rx=v6_rx, v6_tx=v6_tx, v6_rx_nx=v6_rx_nx, **mld(lib))
    np.savez_compressed(os.path.join(OUT, "ref_callers.npz"), **out)
    print("mld:", out["mld_net"].size, "reports")
    np.savez_compressed(os.path.join(OUT, "eth_cases.npz"), **eth(lib))


if __name__ == "__main__":
    main()
