"""The Ethernet front end of the oracle (oracle_batch_eth: the destination filter, the ethertype
dispatch and the IP version checks of pico_ethernet_receive / pico_eth_receive,
modules/pico_ethernet.c:143-235) against the reference's own compiled receive path (CPU).

tests/golden/ref_eth_cases.npz (tests/golden/make_ref_eth.py): 6000 Ethernet frames -- the
datagrams of make_ref_rx.py behind the device's MAC, broadcast, 01:00:5e / 33:33 multicast,
foreign unicast and multicast destinations; ARP, LLDP, unknown ethertypes, IP versions that do not
match the ethertype -- with the reference's L2 decision for every frame and its IP verdict for
the pinned ones.  With oracle/_ref/libref_rx.so present the L2 decisions are re-run live."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_data as G
from tests.test_ref_rx import REF_RX

V_DROP_L2, V_ARP, V_IPV6 = 32, 64, 128


def _desc(c):
    d = np.zeros(c["off"].size, O.DESC_DTYPE)
    d["off"], d["len"] = c["off"], c["avail"]
    return d


def test_oracle_matches_reference_fixture():
    c = G.ref_eth_cases()
    net, l4, v = O.batch_eth(c["buf"], _desc(c), mac=bytes(c["mac"]))
    np.testing.assert_array_equal(v, c["verdict"])
    np.testing.assert_array_equal(net, c["net"])
    np.testing.assert_array_equal(l4, c["l4"])
    l2 = c["l2"]
    # the reference's L2 decision, frame by frame
    assert ((l2 == 0) == (v == V_DROP_L2)).all()
    assert ((l2 == 3) == (v == V_ARP)).all()
    assert ((l2 == 2) == ((v & V_IPV6) != 0)).all()
    assert set(np.unique(l2).tolist()) == {0, 1, 2, 3}
    assert c["pinned"].mean() > 0.9


@pytest.mark.skipif(not os.path.exists(REF_RX), reason="oracle/_ref/libref_rx.so not built (make -C oracle refrx)")
def test_reference_rerun_live_l2():
    R = ctypes.CDLL(REF_RX)
    R.rr_eth_init.argtypes = [ctypes.c_char_p]
    R.rr_eth_rx.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    assert R.rr_init() == 0
    c = G.ref_eth_cases()
    assert R.rr_eth_init(bytes(c["mac"])) == 0
    for i in range(0, c["off"].size, 11):
        o, a = int(c["off"][i]), int(c["avail"][i])
        x = np.ascontiguousarray(c["buf"][o:o + a])
        assert R.rr_eth_rx(x.ctypes.data, a) == c["l2"][i], i
