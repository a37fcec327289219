"""GPU: host-resident descriptor batches (pico_{checksum,ipv4_checksum,ipv6_checksum,
eth_checksum}_batch_host) -- a burst in host memory, chunked H2D / kernel / D2H over two
streams -- against the oracle, with a small staging buffer so every burst spans many chunks;
out-of-bounds and unsorted descriptors; F_WRITE stores written back to host memory."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from picotcp_amd import _lib, batch, synth
from tests import golden_data as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hb():
    h = batch.HostBatch(0, staging_bytes=1 << 20)         # 1 MiB: C2-sized bursts take ~90 chunks
    yield h
    h.close()


def imix_ipv4(n, seed):
    lens = synth.imix_lengths(n, seed)
    buf, net, avail = synth.ipv4_batch(lens, seed=seed, proto=6)
    return buf, batch.make_desc(net, avail)


def test_ipv4_host_rx_tx(hb):
    buf, d = imix_ipv4(100_000, 3)
    on, ol, v = hb.ipv4_checksum_batch(buf, d, flags=_lib.F_TX)
    wn, wl, wv = O.batch_ipv4(buf, d, tx=True)
    np.testing.assert_array_equal(on, wn)
    np.testing.assert_array_equal(ol, wl)
    np.testing.assert_array_equal(v, wv)
    want = buf.copy()
    hb.ipv4_checksum_batch(buf, d, flags=_lib.F_TX | _lib.F_WRITE)     # crc fields stored in host memory
    on, ol, v = hb.ipv4_checksum_batch(buf, d)
    assert (v == 1).all() and (on == 0).all() and (ol == 0).all()
    assert np.count_nonzero(buf != want) <= 4 * d.size
    buf[np.random.default_rng(1).integers(0, buf.size, 500)] ^= 0x20
    on, ol, v = hb.ipv4_checksum_batch(buf, d)
    wn, wl, wv = O.batch_ipv4(buf, d)
    np.testing.assert_array_equal(on, wn)
    np.testing.assert_array_equal(ol, wl)
    np.testing.assert_array_equal(v, wv)


def test_ipv4_host_unsorted_and_out_of_bounds(hb):
    buf, d = imix_ipv4(20_000, 5)
    rng = np.random.default_rng(2)
    d = d[rng.permutation(d.size)]
    d["off"][::97] = buf.size + 5                           # past base_len -> MALFORMED, unread
    d["len"][1::101] = buf.size                             # region past base_len
    on, ol, v = hb.ipv4_checksum_batch(buf, d)
    oob = (d["off"] > buf.size) | (d["len"].astype(np.uint64) > buf.size - np.minimum(d["off"], buf.size))
    assert oob.sum() > 300 and (v[oob] == 8).all() and (on[oob] == 0).all() and (ol[oob] == 0).all()
    wn, wl, wv = O.batch_ipv4(buf, d[~oob])
    np.testing.assert_array_equal(on[~oob], wn)
    np.testing.assert_array_equal(ol[~oob], wl)
    np.testing.assert_array_equal(v[~oob], wv)


def test_ipv6_and_eth_host(hb):
    c6 = G.ipv6_cases()
    ol, v = hb.ipv6_checksum_batch(c6["buf"], G.ipv6_desc(c6))
    np.testing.assert_array_equal(ol, c6["rx_l4"])
    np.testing.assert_array_equal(v, c6["rx_verdict"])
    ce = G.eth_cases()
    on, ol, v = hb.eth_checksum_batch(ce["buf"], G.eth_desc(ce), mac=ce["mac"].tobytes())
    np.testing.assert_array_equal(on, ce["rx_net"])
    np.testing.assert_array_equal(ol, ce["rx_l4"])
    np.testing.assert_array_equal(v, ce["rx_verdict"])


def test_raw_host_with_write(hb):
    n = 30_000
    rng = np.random.default_rng(9)
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 3)[:-1]]).astype(np.uint64)
    buf = synth.random_bytes(77, int(offs[-1]) + int(lens[-1]) + 8)
    d = batch.make_desc(offs, lens, rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32))
    want = O.batch_raw(buf, d, crc_off=2)
    out = hb.checksum_batch(buf, d, crc_off=2, flags=_lib.F_WRITE)
    np.testing.assert_array_equal(out, want)
    has = lens >= 4
    o = offs[has].astype(np.int64)
    np.testing.assert_array_equal((buf[o + 2].astype(np.uint16) << 8) | buf[o + 3], want[has])


def test_frame_larger_than_staging_is_einval(hb):
    buf = np.zeros(3 << 20, np.uint8)
    d = batch.make_desc([0], [2 << 20])
    with pytest.raises(_lib.PicoCsumError) as e:
        hb.checksum_batch(buf, d)
    assert e.value.rc == -_lib.EINVAL


def _packed_small_frames(n, seed):
    """Frames packed back to back (no gaps), 8..200 B, so most start off a 16-byte line and
    chunk boundaries fall inside 16-byte lines shared by two frames."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(8, 200, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64)
    buf = synth.random_bytes(seed, int(offs[-1]) + int(lens[-1]))
    return buf, offs, lens, rng


@pytest.mark.parametrize("shuffle", [False, True])
def test_write_packed_unaligned_and_shuffled(hb, shuffle):
    """F_WRITE on a packed burst (crc at offset 6, as a UDP header) spanning many chunks, in
    ascending order and with the descriptors shuffled: every crc field holds its frame's value
    and no other byte changes."""
    buf, offs, lens, rng = _packed_small_frames(40_000, 71 + shuffle)
    order = rng.permutation(lens.size) if shuffle else np.arange(lens.size)
    d = batch.make_desc(offs[order], lens[order])
    orig = buf.copy()
    want = O.batch_raw(orig, d, crc_off=6)
    out = hb.checksum_batch(buf, d, crc_off=6, flags=_lib.F_WRITE)
    np.testing.assert_array_equal(out, want)
    has = d["len"] >= 8
    o = d["off"][has].astype(np.int64)
    exp = orig.copy()
    exp[o + 6] = (want[has] >> 8).astype(np.uint8)
    exp[o + 7] = (want[has] & 0xFF).astype(np.uint8)
    np.testing.assert_array_equal(buf, exp)


def test_oversized_frame_mid_burst_rx_then_next_call_works(hb):
    """Without F_WRITE a frame too large to stage is found where its chunk would start: -EINVAL
    after the earlier chunks drained, and the context serves the next call."""
    buf, offs, lens, _ = _packed_small_frames(20_000, 6)
    full = np.concatenate([buf, np.zeros(3 << 20, np.uint8)])
    offs2 = np.concatenate([offs[:10_000], [buf.size], offs[10_000:]]).astype(np.uint64)
    lens2 = np.concatenate([lens[:10_000], [2 << 20], lens[10_000:]]).astype(np.uint32)
    with pytest.raises(_lib.PicoCsumError) as e:
        hb.checksum_batch(full, batch.make_desc(offs2, lens2))
    assert e.value.rc == -_lib.EINVAL
    d = batch.make_desc(offs, lens)
    np.testing.assert_array_equal(hb.checksum_batch(full, d), O.batch_raw(full, d))


def test_oversized_frame_mid_burst_with_write_changes_nothing(hb):
    """A frame larger than the staging buffer in the middle of an F_WRITE burst: -EINVAL before
    anything is queued -- no byte of the caller's buffer changes, before or after the return."""
    buf, offs, lens, _ = _packed_small_frames(20_000, 5)
    big = np.zeros(3 << 20, np.uint8)
    full = np.concatenate([buf, big])
    offs = np.concatenate([offs[:10_000], [buf.size], offs[10_000:]]).astype(np.uint64)
    lens = np.concatenate([lens[:10_000], [2 << 20], lens[10_000:]]).astype(np.uint32)
    d = batch.make_desc(offs, lens)
    before = full.copy()
    with pytest.raises(_lib.PicoCsumError) as e:
        hb.checksum_batch(full, d, crc_off=6, flags=_lib.F_WRITE)
    assert e.value.rc == -_lib.EINVAL
    np.testing.assert_array_equal(full, before)
    import time
    time.sleep(0.2)                                  # nothing still in flight lands later
    np.testing.assert_array_equal(full, before)


def test_host_burst_above_2gib(hb):
    """A burst that sits more than 2 GiB into the caller's buffer: its chunks go over
    with rebased descriptors, so the kernels' buffer windows always cover them (no out-of-window
    path); RX, TX and the F_WRITE copy-back against the oracle on the same bytes packed low."""
    small, d = imix_ipv4(30_000, 11)
    hi_off = (9 << 28) + 3                                  # 2.25 GiB + 3 (odd starts)
    big = np.zeros(hi_off + small.size + 64, np.uint8)      # untouched pages stay unallocated
    big[hi_off:hi_off + small.size] = small
    far = d.copy()
    far["off"] += np.uint64(hi_off)
    for fl in (0, _lib.F_TX):
        on, ol, v = hb.ipv4_checksum_batch(big, far, flags=fl)
        wn, wl, wv = O.batch_ipv4(small, d, tx=bool(fl))
        np.testing.assert_array_equal(on, wn)
        np.testing.assert_array_equal(ol, wl)
        np.testing.assert_array_equal(v, wv)
    hb.ipv4_checksum_batch(big, far, flags=_lib.F_TX | _lib.F_WRITE)
    on, ol, v = hb.ipv4_checksum_batch(big, far)
    assert (v == 1).sum() == (wv == 1).sum() and (on[v == 1] == 0).all() and (ol[v == 1] == 0).all()
    del big
