"""The TX side pinned to the frames the compiled reference stack itself emits.

tests/golden/ref_tx_cases.npz (tests/golden/make_ref_tx.py): every IPv4 datagram the CRC=1
reference stack (oracle/_ref/libref_rx.so, compiled unmodified) handed to pico_datalink_send while
it answered SYNs (SYN-ACKs, tcp_send: modules/pico_tcp.c:968-985), sent the data segments of
accepted connections, sent UDP datagrams (crc 0, pico_udp_push: modules/pico_udp.c:120), answered
echo requests and closed ports (pico_icmp4_checksum: modules/pico_icmp4.c:30-41), each behind
pico_ipv4_frame_push's header checksum (modules/pico_ipv4.c:1079).

Here (no GPU): the oracle's TX restatement, run on those datagrams with their crc fields
scrambled, gives exactly the values the reference stored -- on the fixture and on a fresh capture
of the live reference stack (its sequence numbers differ run to run).  tests/test_gpu_ref_tx.py
runs the same datagrams through the GPU batches' F_TX | F_WRITE."""
from __future__ import annotations

import os

import numpy as np
import pytest

from oracle import oracle as O
from picotcp_amd import batch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "ref_tx_cases.npz")
REF_RX = os.path.join(ROOT, "oracle", "_ref", "libref_rx.so")


def fixture():
    c = np.load(GOLDEN)
    return c["buf"].copy(), c["off"].astype(np.uint64), c["len"].astype(np.uint32), c["proto"]


def fields(buf, off, proto):
    """(header crc offset, transport crc offset or -1) of each datagram, from its own header."""
    o = off.astype(np.int64)
    hl = 4 * (buf[o] & 15).astype(np.int64)
    fo = np.select([proto == 6, proto == 17, proto == 1], [16, 6, 2], -1)
    return o + 10, np.where(fo >= 0, o + hl + fo, -1)


def stored(buf, pos):
    return (buf[pos].astype(np.uint16) << 8) | buf[pos + 1]


def scrambled(buf, off, proto, seed):
    """The datagrams with both crc fields overwritten (TX reads them as zero)."""
    b = buf.copy()
    hc, tc = fields(buf, off, proto)
    rng = np.random.default_rng(seed)
    for pos in (hc, tc[tc >= 0]):
        b[pos] = rng.integers(0, 256, pos.size)
        b[pos + 1] = rng.integers(0, 256, pos.size)
    return b


def check_oracle(buf, off, lens, proto):
    desc = batch.make_desc(off, lens)
    hc, tc = fields(buf, off, proto)
    on, ol, v = O.batch_ipv4(scrambled(buf, off, proto, 5), desc, tx=True)
    assert (v == 1).all()
    np.testing.assert_array_equal(on, stored(buf, hc))
    t = tc >= 0
    np.testing.assert_array_equal(ol[t], stored(buf, tc[t]))
    assert (stored(buf, tc[proto == 17]) == 0).all()               # the reference's UDP TX crc is 0


def test_fixture_kinds():
    buf, off, lens, proto = fixture()
    o = off.astype(np.int64)
    assert (proto == 6).sum() >= 40 and (proto == 17).sum() >= 20 and (proto == 1).sum() >= 40
    tcp = o[proto == 6]
    flags = buf[tcp + 33]
    assert ((flags & 0x12) == 0x12).sum() >= 20                     # SYN-ACKs
    assert (lens[proto == 6] > 20 + 4 * (buf[tcp + 32] >> 4)).sum() >= 20   # data segments


def test_oracle_tx_reproduces_reference_frames():
    check_oracle(*fixture())


@pytest.mark.skipif(not os.path.exists(REF_RX), reason="oracle/_ref/libref_rx.so not built here")
def test_oracle_tx_on_live_reference_capture():
    from tests.golden import make_ref_tx as M
    frames = M.capture(seed=int.from_bytes(os.urandom(2), "little"), conns=8)
    buf = np.frombuffer(b"".join(frames), np.uint8).copy()
    lens = np.array([len(f) for f in frames], np.uint32)
    off = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.int64))]).astype(np.uint64)
    proto = np.array([f[9] for f in frames], np.uint8)
    assert (proto == 6).sum() >= 10
    check_oracle(buf, off, lens, proto)
