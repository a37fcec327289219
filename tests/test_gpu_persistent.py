"""GPU: the persistent stream waves (csum_stream_kernel in pico_csum_k_sorted.hip) -- a fixed grid
of waves walking the frame groups, the first one static, the rest claimed from per-XCD heads, each
group streamed or, when it is not back to back, summed by the sorted rounds in the same wave.

Every shape is forced with pico_csum_set_stream_shape at batch sizes where the groups outnumber
the waves several times over (fpw 1 .. 64: up to 8 groups a wave, so the claims, the move to other
XCDs' ranges and the exhaustion path all run), on dense bursts with a share of shuffled descriptors
(groups that fall back to the sorted rounds) and corrupted datagrams, against the oracle bit for
bit: IPv4 RX and TX written in place, IPv6 RX, a mixed IPv4 / IPv6 Ethernet burst.  Repeated
launches and a replayed HIP graph check that the last wave resets the claim counters."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests.test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu

MAC = bytes.fromhex("02005e0a0b0c")


@pytest.fixture(autouse=True)
def _reset_shape():
    yield
    batch.set_stream_shape(0, 0)
    batch.set_launch_override(0, 0, 0)


def shuffle_some(desc, rng, frac):
    """Swap a share of the descriptors with random others: their groups are no longer back to back."""
    d = desc.copy()
    k = int(d.size * frac)
    a = rng.choice(d.size, k, replace=False)
    d[a] = d[rng.permutation(a)]
    return d


def corrupt(buf, desc, rng, frac):
    idx = rng.choice(desc.size, int(desc.size * frac), replace=False)
    off = desc["off"][idx].astype(np.int64) + rng.integers(0, 60, idx.size) % np.maximum(desc["len"][idx], 1)
    buf[off] ^= 0x5A
    return buf


def size_for(wps, fpw):
    """A batch with about 3 groups per persistent wave (256 CUs x 4 SIMDs x wps waves), >= 24000."""
    return max(24000, 1024 * wps * fpw * 3 + 777)


def ipv4_burst(n, seed):
    lens = synth.imix_lengths(n, seed)
    buf, net, avail = synth.ipv4_batch(lens, seed=seed + 1, proto=6, eth=True)
    desc = batch.make_desc(net, avail)
    d_buf = to_dev(buf)
    batch.ipv4_checksum_batch(d_buf, batch.desc_to_device(desc, "cuda:0"), n, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    return d_buf.cpu().numpy(), desc


SHAPES = [(2, 64), (2, 16), (2, 4), (2, 1), (4, 8)]


@pytest.mark.parametrize("wps,fpw", SHAPES)
@pytest.mark.parametrize("shuffled", [0.0, 0.02])
def test_ipv4_rx_tx(wps, fpw, shuffled):
    rng = np.random.default_rng(wps * 100 + fpw + int(shuffled * 1000))
    n = size_for(wps, fpw)
    buf, desc = ipv4_burst(n, 11 + fpw)
    buf = corrupt(buf, desc, rng, 0.01)
    desc = shuffle_some(desc, rng, shuffled)
    batch.set_stream_shape(wps, fpw)
    d_desc = batch.desc_to_device(desc, "cuda:0")
    for _ in range(3):                                    # repeated launches: the counters reset
        on, ol, v = batch.ipv4_checksum_batch(to_dev(buf), d_desc, n)
        torch.cuda.synchronize()
        wn, wl, wv = O.batch_ipv4(buf, desc)
        np.testing.assert_array_equal(v.cpu().numpy(), wv)
        np.testing.assert_array_equal(on.cpu().numpy().view(np.uint16), wn)
        np.testing.assert_array_equal(ol.cpu().numpy().view(np.uint16), wl)
    assert (wv == 1).sum() > n // 2 and (wv != 1).any()
    # TX written in place, then RX of the written bytes
    d_buf = to_dev(buf)
    on, ol, v = batch.ipv4_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    wn, wl, wv = O.batch_ipv4(buf, desc, tx=True)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(on.cpu().numpy().view(np.uint16), wn)
    np.testing.assert_array_equal(ol.cpu().numpy().view(np.uint16), wl)
    got = d_buf.cpu().numpy()
    _, _, rv = O.batch_ipv4(got, desc)
    assert ((wv != 1) | (rv == 1)).all()


@pytest.mark.parametrize("wps,fpw", [(2, 64), (2, 4), (4, 2)])
def test_ipv6_rx(wps, fpw):
    rng = np.random.default_rng(5 + fpw)
    n = size_for(wps, fpw)
    lens = (synth.imix_lengths(n, 3) + 20).astype(np.uint32)
    buf, net, avail, seeds = synth.ipv6_batch(lens, seed=4, proto=6, eth=True)
    desc = batch.make_desc(net, avail, seeds)
    d_buf = to_dev(buf)
    batch.ipv6_checksum_batch(d_buf, batch.desc_to_device(desc, "cuda:0"), n, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    buf = corrupt(d_buf.cpu().numpy(), desc, rng, 0.01)
    desc = shuffle_some(desc, rng, 0.01)
    batch.set_stream_shape(wps, fpw)
    l4, v = batch.ipv6_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), n)
    torch.cuda.synchronize()
    wl, wv = O.batch_ipv6(buf, desc)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(l4.cpu().numpy().view(np.uint16), wl)
    assert (wv == 1).sum() > n // 2


@pytest.mark.parametrize("wps,fpw", [(2, 64), (2, 8), (4, 4)])
def test_ethernet_mixed(wps, fpw):
    rng = np.random.default_rng(9 + fpw)
    n = size_for(wps, fpw)
    lens = synth.imix_lengths(n, 21)
    b4, n4, a4 = synth.ipv4_batch(lens, seed=22, proto=6, eth=True)
    b6, n6, a6, _ = synth.ipv6_batch((lens + 20).astype(np.uint32), seed=23, proto=6, eth=True)
    kinds = rng.integers(0, 2, n)
    buf, st, fl = synth.interleave([(b4, n4 - np.uint64(14), a4 + 14), (b6, n6 - np.uint64(14), a6 + 14)], kinds)
    e = st.astype(np.int64)
    for k, b in enumerate(MAC):
        buf[e + k] = b
    desc = batch.make_desc(st, fl)
    d_buf = to_dev(buf)
    batch.eth_checksum_batch(d_buf, batch.desc_to_device(desc, "cuda:0"), n, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    buf = corrupt(d_buf.cpu().numpy(), desc, rng, 0.01)
    desc = shuffle_some(desc, rng, 0.01)
    batch.set_stream_shape(wps, fpw)
    on, ol, v = batch.eth_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), n, mac=MAC)
    torch.cuda.synchronize()
    wn, wl, wv = O.batch_eth(buf, desc, mac=MAC)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(on.cpu().numpy().view(np.uint16), wn)
    np.testing.assert_array_equal(ol.cpu().numpy().view(np.uint16), wl)


def test_graph_replay():
    """Launches captured in a HIP graph take fixed counter slots; replays must find them reset."""
    n = 30000
    buf, desc = ipv4_burst(n, 40)
    batch.set_stream_shape(2, 2)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc, "cuda:0")
    outs = [tuple(torch.empty(n, dtype=t, device="cuda:0") for t in (torch.int16, torch.int16, torch.uint8))
            for _ in range(3)]
    for o in outs:                                        # warm (outside the capture)
        batch.ipv4_checksum_batch(d_buf, d_desc, n, out=o)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for o in outs:
                batch.ipv4_checksum_batch(d_buf, d_desc, n, out=o)
    torch.cuda.current_stream().wait_stream(s)
    wn, wl, wv = O.batch_ipv4(buf, desc)
    for _ in range(3):
        for o in outs:
            for t in o:
                t.zero_()
        g.replay()
        torch.cuda.synchronize()
        for on, ol, v in outs:
            np.testing.assert_array_equal(v.cpu().numpy(), wv)
            np.testing.assert_array_equal(on.cpu().numpy().view(np.uint16), wn)
            np.testing.assert_array_equal(ol.cpu().numpy().view(np.uint16), wl)
