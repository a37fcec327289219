"""The IPv6 RX dispatch in the oracle (CPU).  By default it is the reference's:
pico_transport_crc_check (stack/pico_socket.c:1919-1958) switches on `net_hdr->proto` read
through a struct pico_ipv4_hdr cast, which for an IPv6 header is byte 9 (the source address's
second byte): byte 9 == 6 -> pico_tcp_checksum (TCP pseudo header), 17 -> the UDP check when
transport bytes 6-7 are non-zero (UDP pseudo header), else none.  PICO_CSUM_F_NXTHDR_DISPATCH
(oracle nxthdr_dispatch) checks by the transport's own protocol instead.  Each default case is
checked against the next-header oracle with the pseudo-header protocol forced through the
descriptor seed (net_len | proto << 16), whose checksum functions are pinned to the compiled
reference callers (tests/test_ref_callers.py); tests/test_ref_rx.py pins the default dispatch
to the reference's own compiled pico_transport_crc_check."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from picotcp_amd import batch, synth


def _one(proto: int, b9: int, corrupt: bool, udp_crc_zero: bool = False):
    buf, net, avail, seeds = synth.ipv6_batch(np.array([200], np.uint32), seed=41 + proto, proto=proto, eth=False)
    d = batch.make_desc(net, avail, seeds)
    o = int(net[0])
    buf[o + 9] = b9
    # a valid checksum for the real protocol (TX oracle), stored as short_be(ret)
    l4, _ = O.batch_ipv6(buf, d, tx=True)
    x = 16 if proto == 6 else 6
    v = 0 if (proto == 17 and udp_crc_zero) else int(l4[0])
    buf[o + 40 + x], buf[o + 40 + x + 1] = v >> 8, v & 0xFF
    if corrupt:
        buf[o + 40 + 30] ^= 0x5A
    return buf, d


def _forced(buf, d, proto):
    f = d.copy()
    f["seed"] = 40 | (proto << 16)
    return O.batch_ipv6(buf, f, nxthdr_dispatch=True)


def test_tcp_checked_only_when_byte9_selects_it():
    for b9 in (6, 17, 99):
        for corrupt in (False, True):
            buf, d = _one(6, b9, corrupt)
            l4, v = O.batch_ipv6(buf, d)
            l4_nx, v_nx = O.batch_ipv6(buf, d, nxthdr_dispatch=True)
            assert v_nx[0] == (batch.V_L4_BAD if corrupt else batch.V_ACCEPT)
            if b9 == 6:                                        # what the next-header check does
                assert (l4[0], v[0]) == (l4_nx[0], v_nx[0])
            elif b9 == 17:                                     # TCP bytes 6-7 (ack) != 0: UDP pseudo header
                fl4, _ = _forced(buf, d, 17)
                assert l4[0] == fl4[0] and l4[0] != 0 and v[0] == batch.V_L4_BAD
            else:                                              # no check at all
                assert (l4[0], v[0]) == (0, batch.V_ACCEPT)


def test_udp_dispatch():
    buf, d = _one(17, 6, False)                                # a valid UDP datagram checked as TCP
    l4, v = O.batch_ipv6(buf, d)
    fl4, _ = _forced(buf, d, 6)
    assert l4[0] == fl4[0] and l4[0] != 0 and v[0] == batch.V_L4_BAD
    for corrupt in (False, True):
        buf, d = _one(17, 17, corrupt)
        assert tuple(x[0] for x in O.batch_ipv6(buf, d)) == \
            tuple(x[0] for x in O.batch_ipv6(buf, d, nxthdr_dispatch=True))
    buf, d = _one(17, 17, True, udp_crc_zero=True)             # crc 0: never checked
    l4, v = O.batch_ipv6(buf, d)
    assert (l4[0], v[0]) == (0, batch.V_ACCEPT)
    buf, d = _one(17, 99, True)
    l4, v = O.batch_ipv6(buf, d)
    assert (l4[0], v[0]) == (0, batch.V_ACCEPT)


def test_icmp6_and_tx_unaffected():
    buf, net, avail, seeds = synth.ipv6_batch(np.array([120], np.uint32), seed=5, proto=58, eth=False, icmp_type=135)
    d = batch.make_desc(net, avail, seeds)
    buf[int(net[0]) + 9] = 6
    assert all((a == b).all() for a, b in zip(O.batch_ipv6(buf, d), O.batch_ipv6(buf, d, nxthdr_dispatch=True)))
    buf, d = _one(6, 17, False)
    assert all((a == b).all() for a, b in zip(O.batch_ipv6(buf, d, tx=True),
                                              O.batch_ipv6(buf, d, tx=True, nxthdr_dispatch=False)))


def test_flag_validation_without_gpu():
    import ctypes

    from picotcp_amd import _lib
    lib = _lib.load()

    def vp(x):
        return ctypes.c_void_p(x)
    # an RX option: rejected with F_TX, before any device work; the IPv4 batch has no such flag
    assert lib.pico_ipv6_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, _lib.F_TX | _lib.F_NXTHDR_DISPATCH,
                                            None, None, None) == -_lib.EINVAL
    assert lib.pico_eth_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, _lib.F_TX | _lib.F_NXTHDR_DISPATCH,
                                           None, None, None, None, None) == -_lib.EINVAL
    assert lib.pico_ipv4_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, _lib.F_NXTHDR_DISPATCH,
                                            None, None, None, None) == -_lib.EINVAL
