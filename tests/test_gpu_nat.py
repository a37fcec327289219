"""GPU: the NAT batch (pico_ipv4_nat_batch_dev: pico_ipv4_nat_outbound / _inbound's frame work,
modules/pico_nat.c:424-545) against the reference-pinned fixture (tests/golden/ref_nat_cases.npz:
the reference's own bytes after NAT on 1310 datagrams) and the oracle on a 64K-datagram IMIX
burst with random records -- every byte of the rewritten buffer, the stored checksums and the
verdicts, on several wave shapes."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests.test_gpu_parity import to_dev
from tests.test_ref_nat import cases

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0, 0, 0)


def run(buf, desc, nat):
    d_buf = to_dev(buf)
    on, ol, v = batch.ipv4_nat_batch(d_buf, to_dev(desc.view(np.uint8)), desc.size, to_dev(nat.view(np.uint8)))
    torch.cuda.synchronize()
    return d_buf.cpu().numpy(), on.cpu().numpy().view(np.uint16), ol.cpu().numpy().view(np.uint16), v.cpu().numpy()


@pytest.mark.parametrize("fpw", [0, 1, 7, 64])
def test_reference_fixture(fpw):
    c = cases()
    if fpw:
        batch.set_launch_override(2, fpw=fpw)
    got, on, ol, v = run(c["buf"], c["desc"], c["nat"])
    wo = c["buf"].copy()
    won, wol, wv = O.batch_ipv4_nat(wo, c["desc"], c["nat"])
    np.testing.assert_array_equal(v, c["verdict"])
    np.testing.assert_array_equal(got, c["want"])       # the reference's bytes, every one
    np.testing.assert_array_equal(on, won)
    np.testing.assert_array_equal(ol, wol)


@pytest.mark.parametrize("seed", [1, 2])
def test_imix_burst_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    n = 65536
    lens = synth.imix_lengths(n, seed)
    buf, net, avail = synth.ipv4_batch(lens, seed=seed, proto=6)
    net = net.astype(np.int64)
    proto = rng.choice(np.array([6, 17, 1, 47], np.uint8), n, p=[0.45, 0.4, 0.1, 0.05])
    buf[net + 9] = proto
    fr = rng.random(n) < 0.03                            # fragments: left for reassembly
    buf[net[fr] + 6] = 0x20
    opt = np.flatnonzero(rng.random(n) < 0.02)           # a header length past the datagram
    buf[net[opt] + 0] = 0x4F
    nat = np.zeros(n, O.NAT_DTYPE)
    nat["addr"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    nat["port"] = rng.integers(0, 1 << 16, n).astype(np.uint16)
    nat["dir"] = rng.choice(np.array([0, 1, 2, 3, 255], np.uint8), n, p=[0.08, 0.5, 0.4, 0.01, 0.01])
    desc = batch.make_desc(net.astype(np.uint64), avail)
    got, on, ol, v = run(buf, desc, nat)
    want = buf.copy()
    won, wol, wv = O.batch_ipv4_nat(want, desc, nat)
    np.testing.assert_array_equal(v, wv)
    np.testing.assert_array_equal(on, won)
    np.testing.assert_array_equal(ol, wol)
    np.testing.assert_array_equal(got, want)
    assert {1, 16, 32}.issubset(set(np.unique(v).tolist()))


@pytest.mark.parametrize("seed", [3, 4])
def test_dense_burst_with_options_vs_oracle(seed):
    """Densely packed datagrams (odd and even starts) of which a few carry IPv4 options: the waves
    without options take the stream-order batch (NAT old port from the head window), a wave
    holding a translated datagram with options falls back to the sorted rounds -- every byte,
    stored checksum and verdict against the oracle."""
    rng = np.random.default_rng(seed)
    n = 16384
    lens = rng.integers(60, 1500, n).astype(np.uint32)
    ihl = np.where(rng.random(n) < 0.004, rng.integers(6, 16, n), 5)
    parts, net, pos = [], np.zeros(n, np.int64), 0
    for h in np.unique(ihl):                            # one packed batch per header length
        sel = np.flatnonzero(ihl == h)
        b, o, _ = synth.ipv4_batch(lens[sel], seed=seed + int(h), proto=6, ihl=int(h))
        ends = np.append(o[1:].astype(np.int64), b.size)
        for k, i in enumerate(sel):
            parts.append((i, b[int(o[k]):int(ends[k])]))
    parts.sort(key=lambda t: t[0])
    for i, fb in parts:                                  # back in datagram order, packed
        net[i] = pos
        pos += fb.size
    buf = np.concatenate([fb for _, fb in parts])
    proto = rng.choice(np.array([6, 17, 1], np.uint8), n, p=[0.5, 0.4, 0.1])
    udp = proto == 17
    buf[net + 9] = proto
    hl = 4 * ihl
    ul = lens - hl                                       # UDP length field for the UDP datagrams
    buf[(net + hl + 4)[udp]] = (ul[udp] >> 8).astype(np.uint8)
    buf[(net + hl + 5)[udp]] = (ul[udp] & 0xFF).astype(np.uint8)
    nat = np.zeros(n, O.NAT_DTYPE)
    nat["addr"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    nat["port"] = rng.integers(0, 1 << 16, n).astype(np.uint16)
    nat["dir"] = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.1, 0.5, 0.4])
    desc = batch.make_desc(net.astype(np.uint64), lens)
    assert (net & 1).any() and (ihl > 5).any()
    for fpw in (0, 64):
        if fpw:
            batch.set_launch_override(2, fpw=fpw)
        got, on, ol, v = run(buf, desc, nat)
        want = buf.copy()
        won, wol, wv = O.batch_ipv4_nat(want, desc, nat)
        np.testing.assert_array_equal(v, wv)
        np.testing.assert_array_equal(on, won)
        np.testing.assert_array_equal(ol, wol)
        np.testing.assert_array_equal(got, want)
