"""The span-stream variant of the sorted kernel (override group 2, unroll 2) on DENSE layouts --
frames in ascending order with gaps of 0-15 bytes, the only waves it takes (others fall back to
the rounds inside the same launch) -- against the oracle: any start alignment, chunks shared by
a frame's tail and the next frame's head, 16-byte frames, frames up to 64 KiB, random and
plausible IPv4 / IPv6 headers (padding behind tot_len, options, extension-header seeds), TX,
and waves mixed with non-dense ones (a frame < 16 B or a wide gap).  Run on an MI355X with
`-m gpu`."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
STREAM_SHAPES = [(2, 8, 64, 2, 2), (2, 8, 9, 2, 1), (2, 8, 64, 1, 2)]   # the last: the rounds, for reference


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0)


def u16(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def dense_layout(rng, n, big: bool, breaks: bool):
    """Frame lengths and starts: 16..40 B (20 %), 41..2000 B, optionally up to 64 KiB (2 %);
    gaps 0..15 B; `breaks` plants a few frames < 16 B and gaps >= 16 B (non-dense waves)."""
    kind = rng.random(n)
    lens = np.where(kind < 0.2, rng.integers(16, 41, n), rng.integers(41, 2001, n)).astype(np.int64)
    if big:
        lens[rng.random(n) < 0.02] = rng.integers(2001, 65536, 1)[0]
    gaps = rng.integers(0, 16, n)
    if breaks:
        sel = rng.random(n) < 0.01
        lens[sel] = rng.integers(0, 16, int(sel.sum()))
        gaps[rng.random(n) < 0.01] = 40
    starts = np.zeros(n, dtype=np.int64)
    first = int(rng.integers(0, 16))
    starts[0] = first
    starts[1:] = first + np.cumsum(lens + gaps)[:-1]
    return starts, lens


@pytest.mark.parametrize("trial", range(6))
def test_stream_raw_dense(trial):
    rng = np.random.default_rng(7000 + trial)
    n = int(rng.integers(100, 6000))
    starts, lens = dense_layout(rng, n, big=trial % 2 == 0, breaks=trial >= 3)
    size = int(starts[-1] + lens[-1] + 32)
    buf = synth.random_bytes(7100 + trial, size)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * (rng.random(n) < 0.5)
    desc = batch.make_desc(starts.astype(np.uint64), lens, seeds)
    crc = int(rng.choice([-1, 0, 2, 10, 16, 6]))
    want = O.batch_raw(buf, desc, crc_off=crc)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc, DEV)
    for shape in STREAM_SHAPES:
        batch.set_launch_override(*shape)
        got = u16(batch.checksum_batch(d_buf, d_desc, n, crc_off=crc))
        np.testing.assert_array_equal(got, want, err_msg=f"trial={trial} shape={shape} crc={crc}")


def dense_datagrams(rng, n, ipv6: bool, breaks: bool):
    starts, lens = dense_layout(rng, n, big=False, breaks=breaks)
    size = int(starts[-1] + lens[-1] + 32)
    buf = synth.random_bytes(int(rng.integers(0, 1 << 30)), size)
    seeds = np.zeros(n, dtype=np.uint32)
    for i in range(n):
        o, L = int(starts[i]), int(lens[i])
        if rng.random() < 0.8 and L >= 40:          # a plausible header; padding behind tot_len at times
            if not ipv6:
                ihl = int(rng.choice([5, 5, 5, 6, 15, 3]))
                buf[o] = 0x40 | ihl
                tot = L - int(rng.integers(0, 12)) if rng.random() < 0.85 else int(rng.integers(0, 65536))
                buf[o + 2], buf[o + 3] = (tot >> 8) & 0xFF, tot & 0xFF
                buf[o + 9] = int(rng.choice([6, 17, 1, 6, 47]))
            else:
                buf[o] = 0x60
                pl = L - 40 - int(rng.integers(0, 12)) if rng.random() < 0.85 else int(rng.integers(0, 65536))
                buf[o + 4], buf[o + 5] = (pl >> 8) & 0xFF, pl & 0xFF
                buf[o + 6] = int(rng.choice([6, 17, 58, 6, 0, 43]))
                if rng.random() < 0.2:
                    seeds[i] = int(rng.choice([48, 40, 56, 136, 2000])) | (int(rng.choice([6, 17, 58])) << 16)
    return buf, batch.make_desc(starts.astype(np.uint64), lens.astype(np.uint32), seeds)


@pytest.mark.parametrize("trial", range(3))
@pytest.mark.parametrize("tx", [False, True])
def test_stream_ipv4_dense(trial, tx):
    rng = np.random.default_rng(7300 + trial)
    n = int(rng.integers(300, 4000))
    buf, desc = dense_datagrams(rng, n, ipv6=False, breaks=trial == 2)
    wn, wl, wv = O.batch_ipv4(buf, desc, tx=tx)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc, DEV)
    for shape in STREAM_SHAPES:
        batch.set_launch_override(*shape)
        net, l4, v = batch.ipv4_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX if tx else 0)
        np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"verdict trial={trial} shape={shape}")
        np.testing.assert_array_equal(u16(net), wn, err_msg=f"net trial={trial} shape={shape}")
        np.testing.assert_array_equal(u16(l4), wl, err_msg=f"l4 trial={trial} shape={shape}")


@pytest.mark.parametrize("trial", range(3))
@pytest.mark.parametrize("tx", [False, True])
def test_stream_ipv6_dense(trial, tx):
    rng = np.random.default_rng(7600 + trial)
    n = int(rng.integers(300, 4000))
    buf, desc = dense_datagrams(rng, n, ipv6=True, breaks=trial == 2)
    wl, wv = O.batch_ipv6(buf, desc, tx=tx)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc, DEV)
    for shape in STREAM_SHAPES:
        batch.set_launch_override(*shape)
        l4, v = batch.ipv6_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX if tx else 0)
        np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"verdict trial={trial} shape={shape}")
        np.testing.assert_array_equal(u16(l4), wl, err_msg=f"l4 trial={trial} shape={shape}")


@pytest.mark.parametrize("tx", [False, True])
def test_stream_eth_burst(tx):
    mac = bytes.fromhex("02005e0a0b0c")
    buf, off, flen, seeds, _ = synth.eth_batch(5000, seed=77, mac=mac)
    desc = batch.make_desc(off, flen, seeds)
    wn, wl, wv = O.batch_eth(buf, desc, mac=None if tx else mac, tx=tx)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc, DEV)
    for shape in STREAM_SHAPES:
        batch.set_launch_override(*shape)
        net, l4, v = batch.eth_checksum_batch(d_buf, d_desc, len(flen), flags=batch.F_TX if tx else 0,
                                              mac=None if tx else mac)
        np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"verdict shape={shape}")
        np.testing.assert_array_equal(u16(net), wn, err_msg=f"net shape={shape}")
        np.testing.assert_array_equal(u16(l4), wl, err_msg=f"l4 shape={shape}")
