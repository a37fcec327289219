"""The Ethernet front end's oracle (oracle_batch_eth) against the committed eth_cases
fixture and against the per-family oracles it dispatches to (CPU only)."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from tests import golden_data as G


def test_fixture_reproduces():
    c = G.eth_cases()
    mac = c["mac"].tobytes()
    on, ol, v = O.batch_eth(c["buf"], G.eth_desc(c), mac=mac)
    np.testing.assert_array_equal(on, c["rx_net"])
    np.testing.assert_array_equal(ol, c["rx_l4"])
    np.testing.assert_array_equal(v, c["rx_verdict"])
    on, ol, v = O.batch_eth(c["buf"], G.eth_desc(c))
    np.testing.assert_array_equal(on, c["rx_net_nomac"])
    np.testing.assert_array_equal(ol, c["rx_l4_nomac"])
    np.testing.assert_array_equal(v, c["rx_verdict_nomac"])
    on, ol, v = O.batch_eth(c["tx_buf"], G.eth_desc(c, rx=False), tx=True)
    np.testing.assert_array_equal(on, c["tx_net"])
    np.testing.assert_array_equal(ol, c["tx_l4"])
    np.testing.assert_array_equal(v, c["tx_verdict"])


def test_every_verdict_class_is_covered():
    c = G.eth_cases()
    v = c["rx_verdict"]
    for bit in (1, 2, 4, 8, 32, 64, 128):
        assert ((v & bit) != 0).any(), bit
    assert (v == (128 | 4)).any() and (v == (128 | 8)).any()     # IPv6 L4_BAD / MALFORMED


def test_dispatch_equals_the_per_family_oracles():
    """An IPv4 frame's outputs equal oracle_batch_ipv4 at +14, an IPv6 frame's equal
    oracle_batch_ipv6 at +14 (| V_IPV6); everything else carries no checksum."""
    c = G.eth_cases()
    d = G.eth_desc(c)
    on, ol, v = O.batch_eth(c["buf"], d)
    et = np.array([(int(c["buf"][o + 12]) << 8) | int(c["buf"][o + 13]) for o in c["off"].astype(int)])
    ver = np.array([int(c["buf"][o + 14]) >> 4 for o in c["off"].astype(int)])
    ok = d["len"] >= 15
    sub = d.copy()
    sub["off"] += 14
    sub["len"] = np.where(d["len"] >= 14, d["len"] - 14, 0)
    n4, l4, v4 = O.batch_ipv4(c["buf"], sub)
    m4 = ok & (et == 0x0800) & (ver == 4)
    np.testing.assert_array_equal(on[m4], n4[m4])
    np.testing.assert_array_equal(ol[m4], l4[m4])
    np.testing.assert_array_equal(v[m4], v4[m4])
    l6, v6 = O.batch_ipv6(c["buf"], sub)
    m6 = ok & (et == 0x86DD) & (ver == 6)
    np.testing.assert_array_equal(ol[m6], l6[m6])
    np.testing.assert_array_equal(v[m6], v6[m6] | 128)
    np.testing.assert_array_equal(on[~m4], 0)
    other = ok & ~m4 & ~m6
    assert set(np.unique(v[other])) <= {32, 64}
    assert (v[other & (et == 0x0806)] == 64).all()
