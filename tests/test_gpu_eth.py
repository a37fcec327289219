"""GPU: the Ethernet front end of the fused RX verify (pico_eth_checksum_batch_dev, one launch
over a mixed IPv4 / IPv6 / ARP / other burst) against the eth_cases fixture and against the
two-launch path (IPv4 and IPv6 batches on the split burst), bit-exact."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from picotcp_amd import _lib, batch, synth
from tests import golden_data as G
from tests.test_gpu_parity import KERNELS, to_dev, u16, use_kernel

pytestmark = pytest.mark.gpu

SORTED = list(KERNELS)


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0)


def u8(t):
    return t.cpu().numpy().view(np.uint8)


@pytest.mark.parametrize("kernel", SORTED)
@pytest.mark.parametrize("mac", [True, False])
def test_eth_rx_vs_fixture(kernel, mac):
    c = G.eth_cases()
    use_kernel(kernel)
    n = c["off"].size
    on, ol, v = batch.eth_checksum_batch(to_dev(c["buf"]), to_dev(G.eth_desc(c).view(np.uint8)), n,
                                         mac=c["mac"].tobytes() if mac else None)
    sfx = "" if mac else "_nomac"
    np.testing.assert_array_equal(u16(on), c["rx_net" + sfx])
    np.testing.assert_array_equal(u16(ol), c["rx_l4" + sfx])
    np.testing.assert_array_equal(u8(v), c["rx_verdict" + sfx])


@pytest.mark.parametrize("kernel", SORTED)
def test_eth_tx_compute_and_write(kernel):
    c = G.eth_cases()
    use_kernel(kernel)
    n = c["off"].size
    d = to_dev(G.eth_desc(c, rx=False).view(np.uint8))
    buf = to_dev(c["tx_buf"])
    on, ol, v = batch.eth_checksum_batch(buf, d, n, flags=_lib.F_TX)
    np.testing.assert_array_equal(u16(on), c["tx_net"])
    np.testing.assert_array_equal(u16(ol), c["tx_l4"])
    np.testing.assert_array_equal(u8(v), c["tx_verdict"])
    batch.eth_checksum_batch(buf, d, n, flags=_lib.F_TX | _lib.F_WRITE)
    back = buf.cpu().numpy()
    # the written frames verify on RX by their own protocol (UDP over IPv4 is sent with crc 0: not
    # verified) -- except IPv6 frames behind headers TX does not walk (a fragment header: RX hands
    # them to reassembly; destination options without an 8-aligned payload: RX discards them) and
    # IPv4 frames with the evil bit (RX discards them after the header check) ...
    _, _, rv = O.batch_eth(back, G.eth_desc(c, rx=False), nxthdr_dispatch=True)
    walked = np.isin(c["kind"], [synth.ETH_KINDS.index(k) for k in ("ipv6_frag", "ipv6_dst_tcp", "ipv4_evil")])
    acc = ((c["tx_verdict"] & 0x7F) == 1) & ~walked
    assert ((rv[acc] & 0x7F) == 1).all()
    # ... fragments got their header checksum only, and are handed to reassembly on RX ...
    frag = (c["tx_verdict"] & 0x7F) == 16
    assert frag.sum() > 10 and ((rv[frag] & 0x7F) == 16).all()
    # ... and only the crc fields changed
    diff = np.flatnonzero(back != c["tx_buf"])
    assert diff.size <= 4 * int(acc.sum()) + 2 * int(frag.sum())
    # the oracle TX on the GPU-written bytes sees the same values again
    on2, ol2, _ = O.batch_eth(back, G.eth_desc(c, rx=False), tx=True)
    np.testing.assert_array_equal(on2, c["tx_net"])
    np.testing.assert_array_equal(ol2, c["tx_l4"])


def test_eth_one_launch_equals_two_launch_path():
    """The single Ethernet launch gives, for every IP frame, what the IPv4 and IPv6 batches
    give on the frames split by ethertype on the host (the pre-Ethernet-step path)."""
    c = G.eth_cases()
    n = c["off"].size
    d = G.eth_desc(c)
    buf = to_dev(c["buf"])
    on, ol, v = (u16(x) if i < 2 else u8(x) for i, x in
                 enumerate(batch.eth_checksum_batch(buf, to_dev(d.view(np.uint8)), n)))
    host = c["buf"]
    et = np.array([(int(host[o + 12]) << 8) | int(host[o + 13]) for o in c["off"].astype(int)])
    ver = np.array([int(host[o + 14]) >> 4 for o in c["off"].astype(int)])
    sub = d.copy()
    sub["off"] += 14
    sub["len"] = np.where(d["len"] >= 14, d["len"] - 14, 0)
    i4 = np.flatnonzero((d["len"] >= 15) & (et == 0x0800) & (ver == 4))
    i6 = np.flatnonzero((d["len"] >= 15) & (et == 0x86DD) & (ver == 6))
    n4, l4, v4 = batch.ipv4_checksum_batch(buf, to_dev(sub[i4].view(np.uint8)), i4.size)
    np.testing.assert_array_equal(on[i4], u16(n4))
    np.testing.assert_array_equal(ol[i4], u16(l4))
    np.testing.assert_array_equal(v[i4], u8(v4))
    l6, v6 = batch.ipv6_checksum_batch(buf, to_dev(sub[i6].view(np.uint8)), i6.size)
    np.testing.assert_array_equal(ol[i6], u16(l6))
    np.testing.assert_array_equal(v[i6], u8(v6) | 128)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_eth_random_bursts_vs_oracle(seed):
    """Fresh seeded bursts, random truncations and ethertype / MAC bytes, vs the oracle."""
    rng = np.random.default_rng(seed)
    buf, off, flen, seeds, _ = synth.eth_batch(int(rng.integers(500, 3000)), seed=100 + seed)
    n = off.size
    d = np.zeros(n, dtype=batch.DESC_DTYPE)
    d["off"], d["len"], d["seed"] = off, flen, seeds
    cut = rng.random(n) < 0.1
    d["len"][cut] = rng.integers(0, 64, int(cut.sum()))
    for o in off[rng.random(n) < 0.05].astype(int):
        buf[o + 12:o + 14] = rng.integers(0, 256, 2)
    mac = bytes.fromhex("02005e0a0b0c")
    dbuf, dd = to_dev(buf), to_dev(d.view(np.uint8))
    for tx in (False, True):
        on, ol, v = batch.eth_checksum_batch(dbuf, dd, n, flags=_lib.F_TX if tx else 0, mac=None if tx else mac)
        wn, wl, wv = O.batch_eth(buf, d, mac=None if tx else mac, tx=tx)
        np.testing.assert_array_equal(u16(on), wn)
        np.testing.assert_array_equal(u16(ol), wl)
        np.testing.assert_array_equal(u8(v), wv)


@pytest.mark.parametrize("kernel", SORTED)
def test_eth_reference_fixture(kernel):
    """The burst whose L2 and IP verdicts come from the reference's own compiled receive path
    (tests/golden/make_ref_eth.py), every kernel variant."""
    c = G.ref_eth_cases()
    d = np.zeros(c["off"].size, batch.DESC_DTYPE)
    d["off"], d["len"] = c["off"], c["avail"]
    use_kernel(kernel)
    net, l4, v = batch.eth_checksum_batch(to_dev(c["buf"]), batch.desc_to_device(d, "cuda:0"), d.size,
                                          mac=bytes(c["mac"]))
    np.testing.assert_array_equal(v.cpu().numpy(), c["verdict"])
    np.testing.assert_array_equal(u16(net), c["net"])
    np.testing.assert_array_equal(u16(l4), c["l4"])

