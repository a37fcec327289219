"""GPU: the reassembly batches on adversarial fragment sets, against the oracle (oracle_ipv4_reassemble,
pinned to the reference's pico_fragments.c by tests/golden/ref_reasm_cases.npz).

Each datagram starts as a valid fragmentation of a random transport (TCP / UDP / other protocol,
fragment payloads a random multiple of 8 bytes), then takes random mutations the reference's
fragment tree has to sort out: retransmissions carrying the same bytes, repeated offsets with
different bytes or a different length, overlaps, holes, a fragment behind the last one, an MF flag
flipped, a truncated descriptor -- arrival order shuffled.  600-1000 datagrams a batch (1 to
over 512 fragments a datagram), under every setting of pico_csum_set_reasm_flat: the launcher's
choice, the flat grid forced (planners with one or two fragments a lane, gather waves, the finish
and its workgroup path for SLOW plans) and one workgroup per datagram.  Every verdict, length,
checksum and reassembled byte is compared."""
from __future__ import annotations

import numpy as np
import pytest

from picotcp_amd import batch
from tests import golden_data as G
from tests.test_gpu_frag import check, layout

pytestmark = pytest.mark.gpu


def _datagram(rng, ident, v6=False):
    """(fragment frames in arrival order, transport length) of one mutated datagram (IPv6: a fixed
    header + a fragment header in front of each payload; byte 9 -- the reference's TCP / UDP
    dispatch -- the protocol or not)."""
    proto = int(rng.choice([6, 17, 0x80] if not v6 else [6, 17, 58]))
    b9 = proto if rng.random() < 0.7 else int(rng.integers(0, 256))
    tl = int(rng.integers(1, 24000))
    fp = 8 * int(rng.integers(1, 200))                    # fragment payload, a multiple of 8
    payload = rng.integers(0, 256, tl, dtype=np.uint8)
    if proto == 17 and tl >= 8:
        payload[4], payload[5] = tl >> 8, tl & 0xFF
    pieces = [(o, payload[o:o + fp]) for o in range(0, tl, fp)]

    def frame(off, data, mf):
        n = data.size
        if v6:
            h = np.zeros(48, np.uint8)
            h[0], h[4], h[5], h[6], h[7] = 0x60, (8 + n) >> 8, (8 + n) & 0xFF, 44, 64
            h[8:24] = [0x20, b9, 0x0d, 0xb8] + [0] * 11 + [1]
            h[24:40] = [0x20, 1, 0x0d, 0xb8] + [0] * 11 + [2]
            om = off | (1 if mf else 0)
            h[40], h[42], h[43] = proto, om >> 8, om & 0xFF
            h[44:48] = [0, 0, ident >> 8, ident & 0xFF]
            return np.concatenate([h, data])
        h = np.zeros(20, np.uint8)
        frag = (off >> 3) | (0x2000 if mf else 0)
        h[0], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9] = (0x45, (20 + n) >> 8, (20 + n) & 0xFF, ident >> 8,
                                                                 ident & 0xFF, frag >> 8, frag & 0xFF, 64, proto)
        h[12:20] = [10, 0, 0, 1, 10, 0, 0, 2]
        return np.concatenate([h, data])

    frags = [frame(o, d, o + d.size < tl) for o, d in pieces]
    for _ in range(int(rng.integers(0, 4))):
        m = int(rng.integers(0, 8))
        k = int(rng.integers(0, len(pieces)))
        o, d = pieces[k]
        if m <= 2:                                        # a retransmission, the same bytes
            frags.append(frame(o, d, o + d.size < tl))
        elif m == 3:                                      # the same offset, different bytes
            frags.append(frame(o, rng.integers(0, 256, d.size, dtype=np.uint8), o + d.size < tl))
        elif m == 4 and d.size > 8:                       # the same offset, shorter
            frags.append(frame(o, d[:d.size - 8], True))
        elif m == 5 and len(frags) > 1:                   # a hole
            frags.pop(int(rng.integers(0, len(frags))))
        elif m == 6:                                      # an overlap (offset 8 into a fragment)
            frags.append(frame(o + 8, payload[o + 8:o + 8 + fp], o + 8 + fp < tl))
        else:                                             # MF flipped on a copy
            frags.append(frame(o, d, not (o + d.size < tl)))
    order = rng.permutation(len(frags)) if rng.random() < 0.8 else np.arange(len(frags))
    return [frags[i] for i in order], tl


def _batch(n, seed, v6=False):
    rng = np.random.default_rng(seed)
    frames, groups, lens = [], [], []
    for g in range(n):
        fs, tl = _datagram(rng, g & 0xFFFF, v6)
        groups.append((len(frames), len(fs)))
        frames.extend(fs)
        lens.append(tl)
    off = np.zeros(len(frames), np.uint64)
    pos = 6
    for i, f in enumerate(frames):
        off[i] = pos
        pos += f.size + int(rng.integers(0, 20))          # gaps of any size: payloads at any alignment
    buf = np.zeros(pos + 16, np.uint8)
    for i, f in enumerate(frames):
        buf[int(off[i]):int(off[i]) + f.size] = f
    flen = np.array([f.size for f in frames], np.uint32)
    if rng.random() < 0.5:                                # a truncated descriptor somewhere
        flen[int(rng.integers(0, len(frames)))] -= 1
    d = G.ipv4_desc(off, flen)
    od, size = layout(lens, shift=8 if v6 else 4, hdr=40 if v6 else 20)
    return buf, d, np.array(groups, np.uint32), od, size


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_fuzz_reassembly(seed, mode):
    """mode: pico_csum_set_reasm_flat -- 0 the launcher's choice, 1 the flat grid forced, 2 one
    workgroup per datagram."""
    buf, d, grp, od, size = _batch(600 + 100 * seed, 900 + seed)
    batch.set_reasm_flat(mode)
    try:
        wl, wv = check(buf, d, grp, od, size)
    finally:
        batch.set_reasm_flat(0)
    assert 0.2 < (wv != 8).mean() < 0.98                 # both outcomes well represented


@pytest.mark.parametrize("nx", [False, True])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("seed", [5, 6])
def test_fuzz_reassembly_ipv6(seed, mode, nx):
    """The same mutations on IPv6 fragments (both TCP / UDP dispatches of the reassembled datagram)."""
    buf, d, grp, od, size = _batch(600 + 100 * seed, 1900 + seed, v6=True)
    batch.set_reasm_flat(mode)
    try:
        wl, wv = check(buf, d, grp, od, size, v6=True, nx=nx)
    finally:
        batch.set_reasm_flat(0)
    assert 0.2 < (wv != 8).mean() < 0.98
