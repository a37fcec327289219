"""GPU: frame layouts that are not one dense span -- each frame in a fixed slot of a driver's ring
(modules/pico_dev_tap.c:63-75 reads one frame per slot-sized buffer), at a jitter inside the slot,
or scattered with random gaps: the waves holding them take the sorted rounds (a round-4 COMPACT
stream over the frames' own lines measured slower and was removed), the dense ones in
the same launch the stream.  IPv4 RX / TX (written in place) / NAT, IPv6, the Ethernet front end,
batches ending inside a workgroup, mixed IPv4 / IPv6 Ethernet bursts, every output and byte against
the oracle."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests.test_gpu_parity import to_dev
from tests.test_gpu_stream import packed_ipv6

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0)


def relayout(buf, desc, rng, slot=2048, jitter=0, gaps=0):
    """The same frames in a fresh buffer (random bytes between them): frame k at k * slot + a
    random 0..jitter (slot > 0), or back to back with random 0..gaps byte gaps (slot == 0)."""
    n = desc.size
    ln = desc["len"].astype(np.int64)
    if slot:
        assert (ln + jitter <= slot).all()
        new = np.arange(n, dtype=np.int64) * slot + rng.integers(0, jitter + 1, n)
    else:
        g = rng.integers(0, gaps + 1, n)
        new = np.concatenate([[0], np.cumsum(ln[:-1] + g[1:])]) + g[0]
    nb = synth.random_bytes(int(rng.integers(0, 1 << 30)), int(new[-1] + ln[-1] + 64))
    for o, L, q in zip(desc["off"].astype(np.int64), ln, new):
        nb[q:q + L] = buf[o:o + L]
    d = desc.copy()
    d["off"] = new.astype(np.uint64)
    return nb, d


def u16(t):
    return t.cpu().numpy().view(np.uint16)


def imix_v4(n, seed, proto=6):
    lens = synth.imix_lengths(n, seed)
    buf, net, avail = synth.ipv4_batch(lens, seed=seed + 1, proto=proto, eth=True)
    return buf, batch.make_desc(net, avail)


@pytest.mark.parametrize("layout", [dict(slot=2048), dict(slot=2048, jitter=15), dict(slot=1600, jitter=3),
                                    dict(slot=0, gaps=4096)])
@pytest.mark.parametrize("fpw", [0, 64, 17])
def test_ipv4_rx_tx_compact(layout, fpw):
    rng = np.random.default_rng(900 + fpw + layout.get("jitter", 0))
    buf, desc = imix_v4(20000, 31 + fpw)
    buf, desc = relayout(buf, desc, rng, **layout)
    if fpw:
        batch.set_launch_override(2, fpw=fpw)
    d_desc = batch.desc_to_device(desc, "cuda:0")
    # TX, written in place
    d_buf = to_dev(buf)
    net, l4, v = batch.ipv4_checksum_batch(d_buf, d_desc, desc.size, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    wn, wl, wv = O.batch_ipv4(buf, desc, tx=True)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(net), wn)
    np.testing.assert_array_equal(u16(l4), wl)
    got = d_buf.cpu().numpy()
    want = buf.copy()
    off = desc["off"].astype(np.int64)
    acc = np.flatnonzero(wv == 1)
    for pos, val in ((off[acc] + 10, wn[acc]), (off[acc] + 36, wl[acc])):
        want[pos], want[pos + 1] = (val >> 8).astype(np.uint8), (val & 0xFF).astype(np.uint8)
    np.testing.assert_array_equal(got, want)
    # RX of the written bytes (all accepted), then with corruption
    got[rng.integers(0, got.size, 3000)] ^= 0x10
    net, l4, v = batch.ipv4_checksum_batch(to_dev(got), d_desc, desc.size)
    wn, wl, wv = O.batch_ipv4(got, desc)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(net), wn)
    np.testing.assert_array_equal(u16(l4), wl)
    assert (wv == 1).sum() > desc.size // 2 and (wv != 1).sum() > 100


@pytest.mark.parametrize("layout", [dict(slot=2048, jitter=7), dict(slot=0, gaps=3000)])
def test_nat_compact(layout):
    rng = np.random.default_rng(77)
    buf, desc = imix_v4(20000, 5)
    buf, desc = relayout(buf, desc, rng, **layout)
    d_buf = to_dev(buf)
    d_desc = batch.desc_to_device(desc, "cuda:0")
    batch.ipv4_checksum_batch(d_buf, d_desc, desc.size, flags=batch.F_TX | batch.F_WRITE)
    before = d_buf.cpu().numpy()
    nat = np.zeros(desc.size, O.NAT_DTYPE)
    nat["addr"] = rng.integers(0, 1 << 32, desc.size, dtype=np.uint64).astype(np.uint32)
    nat["port"] = rng.integers(0, 1 << 16, desc.size).astype(np.uint16)
    nat["dir"] = rng.choice(np.array([0, 1, 2], np.uint8), desc.size, p=[0.1, 0.45, 0.45])
    net, l4, v = batch.ipv4_nat_batch(d_buf, d_desc, desc.size, torch.from_numpy(nat.view(np.uint8)).to("cuda:0"))
    torch.cuda.synchronize()
    want = before.copy()
    wn, wl, wv = O.batch_ipv4_nat(want, desc, nat)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(net), wn)
    np.testing.assert_array_equal(u16(l4), wl)
    np.testing.assert_array_equal(d_buf.cpu().numpy(), want)


@pytest.mark.parametrize("layout", [dict(slot=2048, jitter=9), dict(slot=0, gaps=2500)])
def test_ipv6_compact(layout):
    rng = np.random.default_rng(55)
    buf, desc = packed_ipv6(rng, 20000, 600, 0.002)
    buf, desc = relayout(buf, desc, rng, **layout)
    d_desc = batch.desc_to_device(desc, "cuda:0")
    d_buf = to_dev(buf)
    l4, v = batch.ipv6_checksum_batch(d_buf, d_desc, desc.size, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    wl, wv = O.batch_ipv6(buf, desc, tx=True)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(l4), wl)
    got = d_buf.cpu().numpy()
    for nx in (False, True):
        l4, v = batch.ipv6_checksum_batch(to_dev(got), d_desc, desc.size, flags=batch.F_NXTHDR_DISPATCH if nx else 0)
        wl, wv = O.batch_ipv6(got, desc, nxthdr_dispatch=nx)
        np.testing.assert_array_equal(v.cpu().numpy(), wv)
        np.testing.assert_array_equal(u16(l4), wl)


def test_eth_compact():
    rng = np.random.default_rng(66)
    mac = bytes.fromhex("02005e0a0b0c")
    buf, off, ln, seeds, _ = synth.eth_batch(12000, seed=13, mac=mac)
    buf, desc = relayout(buf, batch.make_desc(off, ln, seeds), rng, slot=2048, jitter=5)
    d_desc = batch.desc_to_device(desc, "cuda:0")
    for fl in (batch.F_TX, 0):
        net, l4, v = batch.eth_checksum_batch(to_dev(buf), d_desc, desc.size, flags=fl, mac=None if fl else mac)
        wn, wl, wv = O.batch_eth(buf, desc, mac=None if fl else mac, tx=bool(fl))
        np.testing.assert_array_equal(v.cpu().numpy(), wv)
        np.testing.assert_array_equal(u16(net), wn)
        np.testing.assert_array_equal(u16(l4), wl)


def test_tiny_and_huge_with_gaps():
    """255 tiny datagrams and one of 20000 bytes per 256, with random gaps: waves whose frames are
    not back to back take the sorted rounds, the others the stream -- same results."""
    rng = np.random.default_rng(3)
    n = 256 * 40
    lens = np.full(n, 40, np.uint32)
    lens[255::256] = 20000
    buf, net, avail = synth.ipv4_batch(lens, seed=8, proto=6, eth=True)
    buf, desc = relayout(buf, batch.make_desc(net, avail), rng, slot=0, gaps=200)
    batch.set_launch_override(2, fpw=64)                # 256-frame workgroups
    for fl in (batch.F_TX, 0):
        net_, l4, v = batch.ipv4_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), n, flags=fl)
        wn, wl, wv = O.batch_ipv4(buf, desc, tx=bool(fl))
        np.testing.assert_array_equal(v.cpu().numpy(), wv)
        np.testing.assert_array_equal(u16(net_), wn)
        np.testing.assert_array_equal(u16(l4), wl)


@pytest.mark.parametrize("n", [1, 3, 63, 65, 255, 257, 1000])
@pytest.mark.parametrize("slot", [0, 2048])
def test_partial_workgroups(n, slot):
    """Batches that end inside a workgroup (waves with no frames take part in its barriers), dense
    and slotted, with invalid and out-of-bounds descriptors mixed in."""
    rng = np.random.default_rng(n + slot)
    buf, desc = imix_v4(n, 40 + n)
    if slot:
        buf, desc = relayout(buf, desc, rng, slot=slot, jitter=3)
    desc["len"][::7] = 10                               # too short: MALFORMED, not part of any range
    desc["off"][5::11] = buf.size + 100                 # out of bounds
    batch.set_launch_override(2, fpw=64)
    # the oracle has no base length: it sees the out-of-bounds frames as empty (MALFORMED, zeros,
    # which the kernel must give them unread)
    odesc = desc.copy()
    odesc["len"][5::11] = 0
    for fl in (batch.F_TX, 0):
        net, l4, v = batch.ipv4_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), n, flags=fl)
        wn, wl, wv = O.batch_ipv4(buf, odesc, tx=bool(fl))
        np.testing.assert_array_equal(v.cpu().numpy(), wv)
        np.testing.assert_array_equal(u16(net), wn)
        np.testing.assert_array_equal(u16(l4), wl)


def mixed_eth(n, seed, mac):
    """IPv4/TCP and IPv6/TCP (or UDP / ICMPv6) Ethernet frames in random order, back to back."""
    rng = np.random.default_rng(seed)
    lens = synth.imix_lengths(n, seed)
    b4, n4, a4 = synth.ipv4_batch(lens, seed=seed + 1, proto=6, eth=True)
    parts = [(b4, n4 - np.uint64(14), a4 + 14)]
    for k, (pr, kw) in enumerate(((6, {}), (17, {}), (58, dict(icmp_type=135)))):
        b6, n6, a6, _ = synth.ipv6_batch((lens + 20).astype(np.uint32), seed=seed + 2 + k, proto=pr, eth=True, **kw)
        parts.append((b6, n6 - np.uint64(14), a6 + 14))
    kinds = rng.choice(4, n, p=[0.5, 0.3, 0.1, 0.1])
    buf, st, fl = synth.interleave(parts, kinds)
    for k, b in enumerate(mac):
        buf[st.astype(np.int64) + k] = b
    buf[st[::97].astype(np.int64) + 23] = 17            # some IPv6 byte-9 = 17 (the reference's UDP dispatch)
    return buf, batch.make_desc(st, fl)


@pytest.mark.parametrize("layout", [None, dict(slot=2048, jitter=1)])
@pytest.mark.parametrize("fpw", [0, 64, 17])
def test_mixed_ethernet_stream(layout, fpw):
    """A mixed IPv4 / IPv6 Ethernet burst in one launch: the IPv6 frames are streamed too (their
    addresses, transport and field by prefixes) -- TX written in place, then RX with both dispatches."""
    mac = bytes.fromhex("02005e0a0b0c")
    rng = np.random.default_rng(fpw + 5)
    buf, desc = mixed_eth(20000, 71 + fpw, mac)
    if layout:
        buf, desc = relayout(buf, desc, rng, **layout)
    if fpw:
        batch.set_launch_override(2, fpw=fpw)
    d_desc = batch.desc_to_device(desc, "cuda:0")
    d_buf = to_dev(buf)
    net, l4, v = batch.eth_checksum_batch(d_buf, d_desc, desc.size, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    wn, wl, wv = O.batch_eth(buf, desc, tx=True)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(net), wn)
    np.testing.assert_array_equal(u16(l4), wl)
    got = d_buf.cpu().numpy()
    got[rng.integers(0, got.size, 2000)] ^= 0x04
    for nx in (False, True):
        net, l4, v = batch.eth_checksum_batch(to_dev(got), d_desc, desc.size, mac=mac,
                                              flags=batch.F_NXTHDR_DISPATCH if nx else 0)
        wn, wl, wv = O.batch_eth(got, desc, mac=mac, nxthdr_dispatch=nx)
        np.testing.assert_array_equal(v.cpu().numpy(), wv)
        np.testing.assert_array_equal(u16(net), wn)
        np.testing.assert_array_equal(u16(l4), wl)
        assert ((wv & 0x7F) == 1).sum() > 15000 and (wv & 128).sum() > 0
