"""GPU: the persistent stream waves for IPv4 descriptor batches (csum_pstream_kernel in
pico_csum_k_sorted.hip, `pico_csum_set_desc_stream(1, wps, fpg)`): a fixed grid of waves streaming
claimed groups back to back, the groups it cannot stream (not back to back) or finish (options, a
field or trailing bytes past the head window) summed by the sorted rounds from the wave's list --
against the oracle and the golden fixtures, at both grid shapes and several group sizes, RX and TX
(written in place), including batches where every group falls back, repeated launches (the claim
counter's reset) and a captured graph."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests import golden_data as G
from tests.test_gpu_parity import DEV, to_dev, u16
from tests.test_gpu_stream import packed_with_tails

pytestmark = pytest.mark.gpu

SHAPES = [(1, 64), (2, 64), (1, 32), (2, 7), (1, 1)]


@pytest.fixture(autouse=True)
def _reset():
    yield
    batch.set_desc_stream(0, 0, 0)
    batch.set_launch_override(0, 0, 0)


def check_ipv4(buf, desc_h, flags=0, d_buf=None):
    n = desc_h.size
    d_buf = to_dev(buf) if d_buf is None else d_buf
    net, l4, v = batch.ipv4_checksum_batch(d_buf, batch.desc_to_device(desc_h, DEV), n, flags=flags)
    torch.cuda.synchronize()
    wn, wl, wv = O.batch_ipv4(buf, desc_h, tx=bool(flags & batch.F_TX))
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(net), wn)
    np.testing.assert_array_equal(u16(l4), wl)
    return d_buf


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("wps,fpg", SHAPES)
def test_golden_fixture(wps, fpg, mode):
    """The IPv4 fixture (valid, corrupted, fragments, evil bit, IHL < 5, bad sources, options,
    truncations), RX and TX, against its expectations; claimed groups and static order."""
    batch.set_desc_stream(mode, wps, fpg)
    cs = G.ipv4_cases()
    desc = batch.desc_to_device(G.ipv4_desc(cs["net"], cs["avail"]), DEV)
    n = cs["net"].size
    for key, buf, flags in (("rx", cs["buf"], 0), ("tx", cs["tx_buf"], batch.F_TX)):
        net, l4, v = batch.ipv4_checksum_batch(to_dev(buf), desc, n, flags=flags)
        np.testing.assert_array_equal(v.cpu().numpy(), cs[f"{key}_verdict"], err_msg=key)
        np.testing.assert_array_equal(u16(net), cs[f"{key}_net"], err_msg=key)
        np.testing.assert_array_equal(u16(l4), cs[f"{key}_l4"], err_msg=key)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("wps,fpg", SHAPES)
def test_c2_imix_rx_with_corruption(wps, fpg, mode):
    """C2's layout (IMIX behind 14-byte gaps), 64K datagrams, 1/37 corrupted."""
    batch.set_desc_stream(mode, wps, fpg)
    lens = synth.imix_lengths(65536, 31 + fpg)
    buf, net_off, avail = synth.ipv4_batch(lens, seed=12 + wps, proto=6, eth=True)
    desc_h = G.ipv4_desc(net_off, avail)
    d_buf = to_dev(buf)
    batch.ipv4_checksum_batch(d_buf, batch.desc_to_device(desc_h, DEV), lens.size, flags=batch.F_TX | batch.F_WRITE)
    h = d_buf.cpu().numpy()
    h[net_off[::37].astype(np.int64) + 25] ^= 0x41
    check_ipv4(h, desc_h)


@pytest.mark.parametrize("wps,fpg", [(1, 64), (2, 64), (1, 17)])
def test_dense_tails_and_options(wps, fpg):
    """Packed datagrams with options, trailing bytes and odd starts: the finish corrects from the
    head window or the group goes on the list for the sorted rounds. RX, TX written in place, RX of
    the written bytes."""
    batch.set_desc_stream(1, wps, fpg)
    rng = np.random.default_rng(5 + wps + fpg)
    buf, desc_h, tail = packed_with_tails(rng, 12000, 40 + fpg, False)
    assert (tail > 0).sum() > 100 and (desc_h["off"] & 1).any()
    d_buf = check_ipv4(buf, desc_h, flags=batch.F_TX | batch.F_WRITE)
    got = d_buf.cpu().numpy()
    wn, wl, wv = O.batch_ipv4(buf, desc_h, tx=True)
    # the written bytes equal what the one-wave-per-group kernel writes
    batch.set_desc_stream(batch.STREAM_OFF)
    d_ref = to_dev(buf)
    batch.ipv4_checksum_batch(d_ref, batch.desc_to_device(desc_h, DEV), desc_h.size, flags=batch.F_TX | batch.F_WRITE)
    np.testing.assert_array_equal(got, d_ref.cpu().numpy())
    batch.set_desc_stream(1, wps, fpg)
    check_ipv4(got, desc_h)
    check_ipv4(buf, desc_h)


@pytest.mark.parametrize("wps,fpg,mode", [(1, 2, 1), (2, 2, 1), (1, 64, 1), (1, 2, 2)])
def test_every_group_falls_back(wps, fpg, mode):
    """No group is back to back: descriptors alternate between two copies of a datagram pool 4 MiB
    apart.  Every group goes on its wave's list; with 2-datagram groups a wave holds ~150 of them,
    so its list fills, the pass runs dry, the sorted rounds empty the list and the next pass starts
    from a fresh claim -- several passes a wave."""
    batch.set_desc_stream(mode, wps, fpg)
    lens = synth.imix_lengths(512, 3)
    pool, net_off, avail = synth.ipv4_batch(lens, seed=4, proto=6, eth=True)
    far = 4 << 20
    buf = np.zeros(far + pool.size, np.uint8)
    buf[:pool.size] = pool
    buf[far:] = pool
    buf[far + net_off[::5].astype(np.int64) + 30] ^= 0x5A       # (the far copy differs a little)
    n = 300000
    k = np.arange(n) % 512
    off = net_off[k].astype(np.uint64) + np.where(np.arange(n) & 1, far, 0).astype(np.uint64)
    check_ipv4(buf, G.ipv4_desc(off, avail[k]))


def test_mixed_dense_and_scattered_groups():
    """Every third group scattered (its datagrams swapped with far ones), the rest back to back."""
    batch.set_desc_stream(1, 1, 64)
    lens = synth.imix_lengths(64 * 900, 8)
    buf, net_off, avail = synth.ipv4_batch(lens, seed=9, proto=6, eth=True)
    desc_h = G.ipv4_desc(net_off, avail)
    idx = np.arange(lens.size)
    for gi in range(0, 900, 3):
        a = gi * 64 + np.arange(0, 64, 2)
        bb = (a + 64 * 450) % lens.size
        idx[a], idx[bb] = bb, a
    check_ipv4(buf, desc_h[idx])


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4097])
def test_small_batches(n):
    """Fewer groups than waves, a partial last group."""
    batch.set_desc_stream(1, 1, 64)
    lens = synth.imix_lengths(n, n)
    buf, net_off, avail = synth.ipv4_batch(lens, seed=n, proto=6, eth=True)
    check_ipv4(buf, G.ipv4_desc(net_off, avail))


def test_out_of_bounds_and_short():
    """Descriptors past base_len and datagrams under 20 bytes inside a streamed group."""
    batch.set_desc_stream(1, 1, 64)
    lens = synth.imix_lengths(6400, 77)
    buf, net_off, avail = synth.ipv4_batch(lens, seed=78, proto=6, eth=True)
    desc_h = G.ipv4_desc(net_off, avail)
    desc_h["len"][5::97] = 11
    desc_h["len"][9::211] = 0
    desc_h["off"][3::301] = np.uint64(1 << 40)
    n = desc_h.size
    net, l4, v = batch.ipv4_checksum_batch(to_dev(buf), batch.desc_to_device(desc_h, DEV), n)
    # the oracle has no bound: past base_len is MALFORMED with zero outputs, as a zero-length one
    ref = desc_h.copy()
    ref["len"][3::301] = 0
    wn, wl, wv = O.batch_ipv4(buf, ref)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(net), wn)
    np.testing.assert_array_equal(u16(l4), wl)
    assert (wv[3::301] == 8).all()


def test_repeated_launches_and_graph():
    """The claim counter is reset by the last wave: 20 launches in a row, then a captured graph
    replayed, each against the oracle."""
    batch.set_desc_stream(1, 1, 64)
    lens = synth.imix_lengths(262144, 2026)
    buf, net_off, avail = synth.ipv4_batch(lens, seed=11, proto=6, eth=True)
    desc_h = G.ipv4_desc(net_off, avail)
    d_buf = to_dev(buf)
    d_desc = batch.desc_to_device(desc_h, DEV)
    batch.ipv4_checksum_batch(d_buf, d_desc, lens.size, flags=batch.F_TX | batch.F_WRITE)
    h = d_buf.cpu().numpy()
    h[net_off[::29].astype(np.int64) + 40] ^= 0x08
    d_buf = to_dev(h)
    wn, wl, wv = O.batch_ipv4(h, desc_h)
    n = lens.size
    outs = [(torch.empty(n, dtype=torch.int16, device=DEV), torch.empty(n, dtype=torch.int16, device=DEV),
             torch.empty(n, dtype=torch.uint8, device=DEV)) for _ in range(3)]
    for k in range(20):
        o = outs[k % 3]
        batch.ipv4_checksum_batch(d_buf, d_desc, n, out=o)
    torch.cuda.synchronize()
    for o in outs:
        np.testing.assert_array_equal(o[2].cpu().numpy(), wv)
        np.testing.assert_array_equal(u16(o[0]), wn)
        np.testing.assert_array_equal(u16(o[1]), wl)
    for o in outs:
        o[2].zero_()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        batch.ipv4_checksum_batch(d_buf, d_desc, n, out=outs[0], stream=s)     # warm-up outside capture
        with torch.cuda.graph(g, stream=s):
            for o in outs:
                batch.ipv4_checksum_batch(d_buf, d_desc, n, out=o, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    for o in outs:
        o[2].zero_()
    for _ in range(4):
        g.replay()
    torch.cuda.synchronize()
    for o in outs:
        np.testing.assert_array_equal(o[2].cpu().numpy(), wv)
        np.testing.assert_array_equal(u16(o[1]), wl)
