"""CPU: the synthetic burst builders the bench and the GPU tests use (picotcp_amd/synth.py) --
slot-ring layout and the interleaving of packed bursts keep every frame's bytes."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from picotcp_amd import batch, synth


def test_slot_layout_matches_packed():
    lens = synth.imix_lengths(3000, 4)
    b, net, av = synth.ipv4_batch(lens, seed=5, proto=6, eth=True)
    s, snet, sav = synth.ipv4_batch(lens, seed=5, proto=6, eth=True, slot=2048)
    assert s.size == 3000 * 2048 and (snet == np.arange(3000) * 2048 + 14).all()
    np.testing.assert_array_equal(sav, av)
    # same headers (the payload bytes differ: the random fill follows the layout)
    for k in range(0, 3000, 97):
        np.testing.assert_array_equal(s[int(snet[k]):int(snet[k]) + 20], b[int(net[k]):int(net[k]) + 20])
    wn, wl, wv = O.batch_ipv4(s, batch.make_desc(snet, sav), tx=True)
    assert (wv == 1).all()


def test_interleave_keeps_frames():
    rng = np.random.default_rng(1)
    parts = []
    for k in range(3):
        ln = rng.integers(1, 300, 500).astype(np.uint32)
        st = np.concatenate([[0], np.cumsum(ln + 3)[:-1]]).astype(np.uint64)
        b = rng.integers(0, 256, int(st[-1] + ln[-1] + 5), dtype=np.uint8)
        parts.append((b, st, ln))
    kinds = rng.integers(0, 3, 1200)
    buf, st, ln = synth.interleave(parts, kinds)
    used = [0, 0, 0]
    for i, k in enumerate(kinds):
        b, s0, l0 = parts[k]
        j = used[k]
        used[k] += 1
        assert ln[i] == l0[j]
        np.testing.assert_array_equal(buf[int(st[i]):int(st[i]) + int(ln[i])], b[int(s0[j]):int(s0[j]) + int(l0[j])])
    assert (st[1:] == st[:-1] + ln[:-1]).all()
