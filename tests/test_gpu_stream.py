"""GPU: the stream-order waves (K4s, `stream_batch` in pico_csum_k_sorted.hip) on densely packed
IPv6 batches -- TCP / UDP / ICMPv6 mixed per datagram, odd and even starts, a few datagrams with
a hop-by-hop header (RX: the extension-header walk, so their waves fall back to the sorted rounds)
-- RX, TX with the fields written in place and RX of the written bytes, against the oracle."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests.test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0, 0, 0)


def packed_ipv6(rng, n, seed, p_hbh):
    """n datagrams, each drawn from one of the per-kind batches, copied back to back."""
    kinds = [dict(proto=6), dict(proto=17), dict(proto=58, icmp_type=128), dict(proto=6, hbh=True, walked=True)]
    pk = np.array([0.5, 0.3, 0.2, 0.0]) * (1 - p_hbh) + np.array([0, 0, 0, p_hbh])
    kind = rng.choice(len(kinds), n, p=pk)
    lens = rng.integers(68, 1500, n).astype(np.uint32)
    frames = [None] * n
    for k, kw in enumerate(kinds):
        sel = np.flatnonzero(kind == k)
        if sel.size == 0:
            continue
        b, o, _, _ = synth.ipv6_batch(lens[sel], seed=seed + k, eth=False, **kw)
        ends = np.append(o[1:].astype(np.int64), b.size)
        for j, i in enumerate(sel):
            frames[i] = b[int(o[j]):int(ends[j])]
    net = np.zeros(n, np.uint64)
    net[1:] = np.cumsum([f.size for f in frames])[:-1]
    buf = np.concatenate(frames)
    avail = np.array([f.size for f in frames], np.uint32)
    return buf, batch.make_desc(net, avail)


@pytest.mark.parametrize("p_hbh", [0.0, 0.003])
@pytest.mark.parametrize("fpw", [0, 64, 17])
def test_dense_ipv6_rx_tx(p_hbh, fpw):
    rng = np.random.default_rng(77 + int(p_hbh * 1000) + fpw)
    n = 20000
    buf, desc = packed_ipv6(rng, n, 500 + fpw, p_hbh)
    assert (desc["off"] & 1).any()
    if fpw:
        batch.set_launch_override(2, fpw=fpw)
    d_desc = batch.desc_to_device(desc, "cuda:0")
    # TX, written in place
    d_buf = to_dev(buf)
    l4, v = batch.ipv6_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    wl, wv = O.batch_ipv6(buf, desc, tx=True)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(l4.cpu().numpy().view(np.uint16), wl)
    # the bytes: the oracle's values stored big-endian at the field of every accepted TCP / UDP /
    # ICMPv6 datagram (offset 16 / 6 / 2 behind the 40-byte header), nothing else changed
    want = buf.copy()
    off = desc["off"].astype(np.int64)
    nh = buf[off + 6]
    fo = np.select([nh == 6, nh == 17, nh == 58], [16, 6, 2], -1)
    w = np.flatnonzero((wv == 1) & (fo >= 0))
    pos = off[w] + 40 + fo[w]
    want[pos] = (wl[w] >> 8).astype(np.uint8)
    want[pos + 1] = (wl[w] & 0xFF).astype(np.uint8)
    got = d_buf.cpu().numpy()
    np.testing.assert_array_equal(got, want)
    # RX of the written datagrams (every TCP / UDP / ICMPv6 one accepted), and of the originals
    for b in (got, buf):
        for nx in (False, True):                     # byte-9 dispatch (the reference's) / next header
            l4, v = batch.ipv6_checksum_batch(to_dev(b), d_desc, n, flags=batch.F_NXTHDR_DISPATCH if nx else 0)
            wl, wv = O.batch_ipv6(b, desc, nxthdr_dispatch=nx)
            np.testing.assert_array_equal(v.cpu().numpy(), wv)
            np.testing.assert_array_equal(l4.cpu().numpy().view(np.uint16), wl)
            if nx and b is got:                      # every written datagram verifies
                assert (wv == 1).sum() >= n - int(p_hbh * n * 3) - 5


def packed_with_tails(rng, n, seed, v6):
    """Densely packed IPv4 (a few with options, IHL 6-15) or IPv6 datagrams of which ~3 % carry
    bytes past the datagram inside their frame (descriptor length > the header's length: Ethernet
    padding, a trailer) -- small datagrams (the frame inside the 64-byte head window) and large ones
    (past it) -- odd and even starts, TCP / UDP / ICMP mixed."""
    small = rng.random(n) < 0.3
    lens = np.where(small, rng.integers(48 if v6 else 28, 60, n), rng.integers(68, 1500, n)).astype(np.uint32)
    if v6:
        lens = np.maximum(lens, 48).astype(np.uint32)
        kinds = [dict(proto=6), dict(proto=17), dict(proto=58, icmp_type=128)]
        kind = rng.choice(3, n, p=[0.5, 0.3, 0.2])
        kind[lens < 60] = 1                               # (TCP needs 20 transport bytes)
    else:
        ihl = np.where(rng.random(n) < 0.02, rng.integers(6, 16, n), 5)
        lens = np.maximum(lens, 4 * ihl + 20).astype(np.uint32)   # (the generator writes a TCP header)
        kind = ihl
    frames = [None] * n
    for k in np.unique(kind):
        sel = np.flatnonzero(kind == k)
        if v6:
            b, o, _, _ = synth.ipv6_batch(lens[sel], seed=seed + int(k), eth=False, **kinds[int(k)])
        else:
            b, o, _ = synth.ipv4_batch(lens[sel], seed=seed + int(k), proto=6, ihl=int(k))
        ends = np.append(o[1:].astype(np.int64), b.size)
        for j, i in enumerate(sel):
            frames[i] = b[int(o[j]):int(ends[j])]
    if not v6:                                            # TCP / UDP / ICMP (UDP length set)
        proto = rng.choice(np.array([6, 17, 1], np.uint8), n, p=[0.5, 0.3, 0.2])
        for i in range(n):
            f = frames[i]
            hl = 4 * int(f[0] & 0x0F)
            if proto[i] == 6 and f.size - hl < 20:
                continue
            f[9] = proto[i]
            if proto[i] == 17 and f.size >= hl + 8:
                ul = int(f.size - hl)
                f[hl + 4], f[hl + 5] = ul >> 8, ul & 0xFF
    tail = np.where(rng.random(n) < 0.03, rng.integers(1, 40, n), 0)
    parts = [np.concatenate([frames[i], rng.integers(0, 256, int(tail[i]), dtype=np.uint8)]) for i in range(n)]
    net = np.zeros(n, np.uint64)
    net[1:] = np.cumsum([f.size for f in parts])[:-1]
    avail = np.array([f.size for f in parts], np.uint32)
    return np.concatenate(parts), batch.make_desc(net, avail), tail


def behind_ethernet(buf, desc, v6):
    """Each datagram of a packed batch behind a 14-byte Ethernet header (broadcast destination)."""
    off = desc["off"].astype(np.int64)
    ln = desc["len"].astype(np.int64)
    eth = np.frombuffer(b"\xff" * 6 + b"\x02\x00\x00\x00\x00\x01" + (b"\x86\xdd" if v6 else b"\x08\x00"), np.uint8)
    parts = [np.concatenate([eth, buf[o:o + n]]) for o, n in zip(off, ln)]
    net = np.zeros(off.size, np.uint64)
    net[1:] = np.cumsum([f.size for f in parts])[:-1]
    return np.concatenate(parts), batch.make_desc(net, (ln + 14).astype(np.uint32))


@pytest.mark.parametrize("v6", [False, True])
@pytest.mark.parametrize("fpw", [0, 64])
@pytest.mark.parametrize("eth", [False, True])
def test_dense_tails_and_options(v6, fpw, eth):
    """The stream takes its regions' ends at the frames' ends and (IPv4) the transport start as if
    there were no options; the finish corrects both from the head window -- or, when the options,
    the field or the bytes past the datagram lie beyond it, the wave falls back to the sorted rounds.
    RX and TX (written in place, then RX of the written bytes) against the oracle."""
    rng = np.random.default_rng(91 + fpw + v6)
    n = 12000
    buf, desc, tail = packed_with_tails(rng, n, 300 + fpw, v6)
    if eth:                                              # MODE 3: the Ethernet front end
        buf, desc = behind_ethernet(buf, desc, v6)
    assert (tail > 0).sum() > 100 and (desc["off"] & 1).any()
    if fpw:
        batch.set_launch_override(2, fpw=fpw)
    d_desc = batch.desc_to_device(desc, "cuda:0")
    if eth:
        run = batch.eth_checksum_batch
        ref = lambda b, **kw: O.batch_eth(b, desc, **kw)
    else:
        run = batch.ipv6_checksum_batch if v6 else batch.ipv4_checksum_batch
        ref = (lambda b, **kw: (None,) + O.batch_ipv6(b, desc, **kw)) if v6 else (lambda b, **kw: O.batch_ipv4(b, desc, **kw))
    d_buf = to_dev(buf)
    out = run(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    want = ref(buf, tx=True)
    np.testing.assert_array_equal(out[-1].cpu().numpy(), want[-1])
    np.testing.assert_array_equal(out[-2].cpu().numpy().view(np.uint16), want[-2])
    if not v6 or eth:
        np.testing.assert_array_equal(out[0].cpu().numpy().view(np.uint16), want[0])
    got = d_buf.cpu().numpy()
    for b in (got, buf):
        out = run(to_dev(b), d_desc, n)
        want = ref(b)
        np.testing.assert_array_equal(out[-1].cpu().numpy(), want[-1])
        np.testing.assert_array_equal(out[-2].cpu().numpy().view(np.uint16), want[-2])
        if b is got:                                     # the written batch verifies
            assert ((want[-1] & 0x7F) == 1).sum() > n // 2
