"""The fused RX verdicts of the oracle against the reference's own compiled RX path (CPU).

tests/golden/ref_rx_cases.npz (made by tests/golden/make_ref_rx.py) holds 5000 IPv4 and 5000
IPv6 datagrams with the verdict the reference's pico_ipv4_process_in / pico_ipv6_extension_headers
/ pico_transport_crc_check produce on them, compiled unmodified from /root/reference
(oracle/_ref/libref_rx.so, oracle/ref_rx_wrap.c + ref_rx_driver.c): the evil bit, IHL < 5,
invalid sources, fragments (IPv4 MF / offset, IPv6 fragment headers), extension-header chains
the reference discards, and the byte-9 transport dispatch.  Rows with pinned == False are where
the reference would read past its buffer or never terminate: restatement only (MALFORMED).
When oracle/_ref/libref_rx.so is present (it is built here and travels prebuilt), the
reference is also re-run live on every pinned row."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_data as G

REF_RX = os.path.join(os.path.dirname(O.HERE), "oracle", "_ref", "libref_rx.so")


def _desc(c, p):
    d = np.zeros(c[p + "_off"].size, O.DESC_DTYPE)
    d["off"], d["len"] = c[p + "_off"], c[p + "_avail"]
    return d


def test_oracle_ipv4_matches_reference_fixture():
    c = G.ref_rx_cases()
    on, ol, v = O.batch_ipv4(c["v4_buf"], _desc(c, "v4"))
    np.testing.assert_array_equal(v, c["v4_verdict"])
    np.testing.assert_array_equal(on, c["v4_net"])
    np.testing.assert_array_equal(ol, c["v4_l4"])
    assert c["v4_pinned"].mean() > 0.95
    kinds = set(np.unique(c["v4_verdict"][c["v4_pinned"]]).tolist())
    assert kinds == {1, 2, 4, 8, 16}, kinds


def test_oracle_ipv6_matches_reference_fixture():
    c = G.ref_rx_cases()
    l4, v = O.batch_ipv6(c["v6_buf"], _desc(c, "v6"))
    np.testing.assert_array_equal(v, c["v6_verdict"])
    np.testing.assert_array_equal(l4, c["v6_l4"])
    pin = c["v6_pinned"]
    assert pin.mean() > 0.8
    assert set(np.unique(c["v6_verdict"][pin]).tolist()) == {1, 4, 8, 16}
    # transports reached behind extension headers the kernel had to walk
    assert ((c["v6_net_len"] > 40) & (c["v6_verdict"] <= 4) & pin).sum() > 100


def test_ipv6_walk_reference_hangs_and_overreads_are_malformed():
    """Inputs the reference cannot run (it loops forever or reads past the buffer): the
    restatement's WALK_BAD, a MALFORMED verdict."""
    def dgram(first, ext, tail=b"", plen=None):
        h = bytearray(40)
        h[0], h[6] = 0x60, first
        body = bytes(ext) + tail
        pl = len(body) if plen is None else plen
        h[4], h[5] = pl >> 8, pl & 0xFF
        return np.frombuffer(bytes(h) + body, np.uint8).copy()
    # hop-by-hop PadN with length 254: optlen (uint8)(254 + 2) = 0, pico_ipv6_process_hopbyhop never ends
    assert O.ipv6_walk(dgram(0, [6, 0, 1, 254, 0, 0, 0, 0], bytes(20)))[0] == O.WALK_BAD
    # destination options: the same in pico_ipv6_process_destopt
    assert O.ipv6_walk(dgram(60, [6, 0, 1, 254, 0, 0, 0, 0], bytes(20)))[0] == O.WALK_BAD
    # the sequence check's (uint8)IPV6_OPTLEN(31) = 0 revisits a header that names itself
    assert O.ipv6_walk(dgram(60, [60, 31] + [0] * 254, bytes(20)))[0] == O.WALK_BAD
    # a header running past the frame
    assert O.ipv6_walk(dgram(0, [6, 3, 1, 0]))[0] == O.WALK_BAD
    # well-formed: hop-by-hop (router alert, MLD) + destination options -> TCP at 56
    k, nl, pr = O.ipv6_walk(dgram(0, [60, 0, 5, 2, 0, 0, 1, 0] + [6, 0, 1, 4, 0, 0, 0, 0], bytes(24)))
    assert (k, nl, pr) == (O.WALK_PROTO, 56, 6)
    # a fragment header -> reassembly
    assert O.ipv6_walk(dgram(44, [17, 0, 0, 9, 1, 2, 3, 4], bytes(16)))[0] == O.WALK_FRAG
    for d in (dgram(0, [6, 0, 1, 254, 0, 0, 0, 0], bytes(20)),):
        desc = np.zeros(1, O.DESC_DTYPE)
        desc["len"] = d.size
        assert O.batch_ipv6(d, desc)[1][0] == 8


@pytest.mark.skipif(not os.path.exists(REF_RX), reason="oracle/_ref/libref_rx.so not built (make -C oracle refrx)")
def test_reference_rerun_live_on_pinned_rows():
    """The compiled reference again, on a sample of the pinned rows (catches a stale fixture)."""
    R = ctypes.CDLL(REF_RX)
    R.rr_ipv4_rx.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    R.rr_ipv4_link.argtypes = [ctypes.c_uint32]
    R.rr_ipv6_rx.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
    assert R.rr_init() == 0
    for i in range(1, 9):
        R.rr_ipv4_link(int.from_bytes(bytes([192, 168, 7, i]), "little"))
    c = G.ref_rx_cases()
    for i in np.flatnonzero(c["v4_pinned"])[::7]:
        o, a = int(c["v4_off"][i]), int(c["v4_avail"][i])
        x = np.ascontiguousarray(c["v4_buf"][o:o + a])
        r = R.rr_ipv4_rx(x.ctypes.data, a)
        want = int(c["v4_verdict"][i])
        if r & 1:
            assert want == 16
        elif r & 2:
            assert want == (1 if (((r >> 8) & 0xFF) not in (6, 17) or r & 4) else 4)
        else:
            assert want in (2, 8) and (want == 2) == (not (r & 16) and want != 8)
    for i in np.flatnonzero(c["v6_pinned"])[::7]:
        o, a = int(c["v6_off"][i]), int(c["v6_avail"][i])
        x = np.ascontiguousarray(c["v6_buf"][o:o + a])
        nl, pr = ctypes.c_uint32(0), ctypes.c_uint32(0)
        r = R.rr_ipv6_rx(x.ctypes.data, a, ctypes.byref(nl), ctypes.byref(pr))
        want = int(c["v6_verdict"][i])
        if (r & 3) == 0:
            assert want == 8
        elif (r & 3) == 2:
            assert want == 16
        elif pr.value in (6, 17):
            assert want == (1 if r & 4 else 4)
