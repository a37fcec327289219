#!/usr/bin/env python3
"""Generates tests/golden/c_abi_burst.bin, the fixture of the C-language ABI check
(tests/c_abi/abi_check.c).  Test infrastructure: expected values
come from the oracle (oracle/pico_csum_oracle.c, pinned to the reference's
stack/pico_frame.c by tests/test_oracle.py).

Layout (little-endian):
  "PCSA" u32 version=1
  u32 n            datagrams of a mixed IPv4 burst (IMIX {64,576,1500}, TCP / UDP / ICMP)
  u32 buf_len      bytes of the burst (14 B Ethernet header in front of each datagram)
  u8  buf[buf_len] the burst, every crc field zero
  desc[n]          struct pico_csum_desc {u64 off; u32 len; u32 seed}
  u16 tx_net[n], u16 tx_l4[n], u8 tx_verdict[n]     pico_ipv4_checksum_batch_dev(F_TX)
  u16 rx_net[n], u16 rx_l4[n], u8 rx_verdict[n]     RX verify after the TX write, with
                                                    every 7th datagram's last byte +1
  u32 u_n, u32 u_len, u64 u_seed                    uniform host batch: frames = splitmix64
  u16 u_out[u_n]                                    bytes (picotcp_amd/synth.py), packed
"""
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from oracle import oracle as O  # noqa: E402
from picotcp_amd import synth  # noqa: E402


def main():
    lens = synth.imix_lengths(384, 77)
    parts, nets, avails, off = [], [], [], 0
    for i, proto in enumerate((6, 17, 1)):
        sel = lens[i::3]
        b, net, av = synth.ipv4_batch(sel, seed=200 + i, proto=proto, eth=True)
        parts.append(b)
        nets.append(net + np.uint64(off))
        avails.append(av)
        off += b.size
    buf = np.concatenate(parts)
    net = np.concatenate(nets)
    avail = np.concatenate(avails)
    n = net.size
    desc = np.zeros(n, dtype=O.DESC_DTYPE)
    desc["off"], desc["len"] = net, avail
    tx = O.batch_ipv4(buf, desc, tx=True)
    # the TX write as the stack does it (hdr->crc = short_be(ret) etc.), via the oracle's
    # own expectations: write them, then verify
    w = buf.copy()
    for i in range(n):
        o, hl = int(net[i]), 4 * (int(w[int(net[i])]) & 15)
        if tx[2][i] != 1:
            continue
        w[o + 10], w[o + 11] = tx[0][i] >> 8, tx[0][i] & 0xFF
        proto = int(w[o + 9])
        if proto == 6:
            p = o + hl + 16
        elif proto == 1:
            p = o + hl + 2
        else:
            p = o + hl + 6
        w[p], w[p + 1] = tx[1][i] >> 8, tx[1][i] & 0xFF
    for i in range(0, n, 7):
        last = int(net[i]) + int(avail[i]) - 1
        w[last] = (int(w[last]) + 1) & 0xFF
    rx = O.batch_ipv4(w, desc, tx=False)
    u_n, u_len, u_seed = 1024, 1500, 0x1500
    frames = synth.uniform_batch(u_n, u_len, seed=u_seed)
    u_out = O.batch_uniform(frames, u_len, u_len, u_n)

    out = bytearray(b"PCSA" + struct.pack("<III", 1, n, buf.size))
    out += buf.tobytes() + desc.tobytes()
    for a in (*tx, *rx):
        out += np.ascontiguousarray(a).tobytes()
    out += struct.pack("<IIQ", u_n, u_len, u_seed) + u_out.tobytes()
    path = os.path.join(HERE, "c_abi_burst.bin")
    with open(path, "wb") as f:
        f.write(out)
    print(f"{path}: {len(out)} bytes, {n} datagrams, tx accept {int((tx[2] == 1).sum())}, "
          f"rx accept {int((rx[2] == 1).sum())}")


if __name__ == "__main__":
    main()
