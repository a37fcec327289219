"""IPv4 forwarding step (the ad-hoc incremental update of
modules/pico_ipv4.c:1547-1556): ttl - 1 in place, expired at 0, else the reference's
`hdr->crc++` (a native little-endian increment of the stored big-endian field).

Parity unpinned: pico_ipv4_forward is static in pico_ipv4.c, which needs the whole
stack, and the reference has no test or fixture for it; the oracle restates the three
lines and is checked here against a second, independent restatement."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from picotcp_amd import batch, synth

V_ACCEPT, V_MALFORMED, V_EXPIRED = 1, 8, 16


def headers(n: int, seed: int):
    """n IPv4 headers packed with 0..3 byte gaps (odd alignments), edge TTL / crc values."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(20, 90, n).astype(np.uint32)
    lens[:5] = [19, 0, 20, 20, 21]                    # too short, empty, minimal
    gaps = rng.integers(0, 4, n).astype(np.uint64)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens.astype(np.uint64) + gaps)[:-1]
    buf = synth.random_bytes(seed, int(off[-1]) + int(lens[-1]) + 8)
    o = off.astype(np.int64)
    ttl = rng.integers(0, 256, n)
    ttl[5:13] = [0, 1, 2, 255, 1, 0, 128, 2]
    buf[o + 8] = ttl.astype(np.uint8)
    crc = rng.integers(0, 1 << 16, n)
    crc[13:19] = [0xFFFF, 0x00FF, 0xFF00, 0, 0xFEFF, 0x0100]
    buf[o + 10] = (crc >> 8).astype(np.uint8)         # stored big-endian (short_be)
    buf[o + 11] = (crc & 0xFF).astype(np.uint8)
    return buf, batch.make_desc(off, lens)


def restated(buf: np.ndarray, desc: np.ndarray):
    """Independent restatement of pico_ipv4.c:1547-1556 (Python ints)."""
    out = buf.copy()
    v = np.zeros(desc.size, np.uint8)
    for i, (off, ln, _) in enumerate(desc.tolist()):
        if ln < 20:
            v[i] = V_MALFORMED
            continue
        ttl = (int(out[off + 8]) - 1) & 0xFF          # hdr->ttl = (uint8_t)(hdr->ttl - 1)
        out[off + 8] = ttl
        if ttl < 1:
            v[i] = V_EXPIRED
            continue
        c = (int(out[off + 10]) | int(out[off + 11]) << 8) + 1   # hdr->crc++ on a LE host
        out[off + 10] = c & 0xFF
        out[off + 11] = (c >> 8) & 0xFF
        v[i] = V_ACCEPT
    return out, v


def test_oracle_forward_matches_restatement():
    buf, desc = headers(3000, 7)
    want_buf, want_v = restated(buf, desc)
    got = buf.copy()
    v = O.batch_ipv4_forward(got, desc)
    np.testing.assert_array_equal(v, want_v)
    np.testing.assert_array_equal(got, want_buf)
    assert (want_v == V_EXPIRED).sum() > 0 and (want_v == V_MALFORMED).sum() == 2


def test_forward_keeps_valid_headers_valid():
    """The reference's crc++ is the one's-complement update for -1 on the TTL byte
    (+0x0100 on the checksum, the carry out of the first stored byte landing in the
    second as the end-around carry): a valid header stays valid after the step."""
    lens = np.full(2000, 64, dtype=np.uint32)
    buf, net, avail = synth.ipv4_batch(lens, seed=3, proto=17, eth=True)
    desc = batch.make_desc(net, avail)
    for o in net.astype(np.int64):
        h = buf[o:o + 20].copy()
        h[10:12] = 0
        c = O.checksum(h)
        buf[o + 10], buf[o + 11] = c >> 8, c & 0xFF
    v = O.batch_ipv4_forward(buf, desc)
    assert (v == V_ACCEPT).all()                       # ttl 64 -> 63
    for o in net.astype(np.int64):
        assert O.checksum(buf[o:o + 20]) == 0


@pytest.mark.gpu
def test_gpu_forward_matches_oracle():
    import torch
    for seed in (1, 2, 3):
        buf, desc = headers(20000, seed)
        want_buf = buf.copy()
        want_v = O.batch_ipv4_forward(want_buf, desc)
        d_buf = torch.from_numpy(buf).to("cuda:0")
        v = batch.ipv4_forward_batch(d_buf, batch.desc_to_device(desc, "cuda:0"), desc.size)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(v.cpu().numpy(), want_v)
        np.testing.assert_array_equal(d_buf.cpu().numpy(), want_buf)


@pytest.mark.gpu
def test_gpu_forward_out_of_bounds_untouched():
    import torch
    buf = synth.random_bytes(4, 4096)
    desc = batch.make_desc([0, 4090, 1 << 40, 100], [20, 20, 20, 20])
    want = buf.copy()
    wv = O.batch_ipv4_forward(want, desc[[0, 3]])
    d_buf = torch.from_numpy(buf).to("cuda:0")
    v = batch.ipv4_forward_batch(d_buf, batch.desc_to_device(desc, "cuda:0"), 4).cpu().numpy()
    np.testing.assert_array_equal(v, [wv[0], V_MALFORMED, V_MALFORMED, wv[1]])
    np.testing.assert_array_equal(d_buf.cpu().numpy(), want)
