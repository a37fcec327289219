"""The reference's own compiled checksum callers (tests/golden/ref_callers.npz, made by
make_ref_callers.py from pico_tcp.c / pico_udp.c / pico_icmp6.c / pico_mld.c) against
the fixtures the GPU tests use, the C oracle, and libpicocsum's host helpers (CPU only)."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from oracle import oracle as O
from picotcp_amd import _lib
from tests import golden_data as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_CALLERS = os.path.join(ROOT, "oracle", "_ref", "libref_callers.so")


def test_fixture_rows_match_the_ipv4_ipv6_expectations():
    rc, c4, c6 = G.ref_callers(), G.ipv4_cases(), G.ipv6_cases()
    assert rc["v4_rx"].size == c4["net"].size and rc["v6_rx"].size == c6["net"].size
    for got, exp in ((rc["v4_rx"], c4["rx_l4"]), (rc["v4_tx"], c4["tx_l4"]),
                     (rc["v6_rx"], c6["rx_l4"]), (rc["v6_tx"], c6["tx_l4"])):
        m = got >= 0
        assert m.sum() > 250
        np.testing.assert_array_equal(got[m], exp[m].astype(np.int32))


def test_oracle_fused_batches_match_the_reference_callers():
    rc, c4, c6 = G.ref_callers(), G.ipv4_cases(), G.ipv6_cases()
    _, l4, _ = O.batch_ipv4(c4["buf"], G.ipv4_desc(c4["net"], c4["avail"]))
    m = rc["v4_rx"] >= 0
    np.testing.assert_array_equal(l4[m].astype(np.int32), rc["v4_rx"][m])
    _, l4, _ = O.batch_ipv4(c4["tx_buf"], G.ipv4_desc(c4["net"], c4["avail"]), tx=True)
    m = rc["v4_tx"] >= 0
    np.testing.assert_array_equal(l4[m].astype(np.int32), rc["v4_tx"][m])
    for buf, key, tx in ((c6["buf"], "v6_rx", False), (c6["tx_buf"], "v6_tx", True)):
        l4, _ = O.batch_ipv6(buf, G.ipv6_desc(c6), tx=tx)
        m = rc[key] >= 0
        np.testing.assert_array_equal(l4[m].astype(np.int32), rc[key][m])


def mld_expected_by_seed(lib, rc, tx: bool) -> np.ndarray:
    """pico_mld_checksum through libpicocsum's layer 1: seed = pico_ipv6_pseudo_partial over
    (src, dst, 58, len - 8), then the report region (transport + 8, len - 8)."""
    buf = rc["mld_buf"].copy()
    out = np.zeros(rc["mld_net"].size, dtype=np.uint16)
    for i, (o, size) in enumerate(zip(rc["mld_net"].astype(int), rc["mld_size"].astype(int))):
        rep = buf[o + 48:o + size].copy()
        if tx:
            rep[2:4] = 0
        h = buf[o:o + 40]
        seed = lib.pico_ipv6_pseudo_partial(h[8:24].ctypes.data, h[24:40].ctypes.data, 58, rep.size)
        s = lib.pico_checksum_partial(seed, rep.ctypes.data, rep.size)
        out[i] = finalize(s)
    return out


def finalize(s: int) -> int:
    """stack/pico_frame.c:301-307"""
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    c = ~s & 0xFFFF
    return ((c >> 8) | (c << 8)) & 0xFFFF


@pytest.mark.parametrize("tx", [False, True])
def test_mld_checksum_via_ipv6_pseudo_seed(tx):
    rc = G.ref_callers()
    got = mld_expected_by_seed(_lib.load(), rc, tx)
    np.testing.assert_array_equal(got.astype(np.int32), rc["mld_tx" if tx else "mld_rx"])


@pytest.mark.skipif(not os.path.exists(REF_CALLERS), reason="oracle/_ref/libref_callers.so not built here")
def test_fixture_regenerates_from_the_reference_build():
    """The committed values are what the reference build returns now (a sample)."""
    lib = ctypes.CDLL(REF_CALLERS)
    lib.rc_checksum.restype = ctypes.c_int
    lib.rc_checksum.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_int]
    rc = G.ref_callers()
    for i in range(0, rc["mld_net"].size, 7):
        o, size = int(rc["mld_net"][i]), int(rc["mld_size"][i])
        d = np.ascontiguousarray(rc["mld_buf"][o:o + size])
        assert lib.rc_checksum(5, d.ctypes.data, size, 40, size - 40, 0) == rc["mld_rx"][i]
        assert lib.rc_checksum(5, d.ctypes.data, size, 40, size - 40, 1) == rc["mld_tx"][i]
