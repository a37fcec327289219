"""IPv4 reassembly restatement (oracle_ipv4_reassemble) against the reference's own unit-test
expectations for pico_fragments_check_complete / pico_fragments_reassemble /
pico_ipv4_process_frag (test/unit/modunit_pico_fragments.c:223-347, 825-935, 1064-1160,
re-expressed as fragment frames: libcheck is not available to run them) and against an
independent Python restatement on seeded fragment sets (CPU only)."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from picotcp_amd import synth
from tests import golden_data as G

MF = 0x2000


def frame(payload: int, frag: int, proto: int = 0x80, ident: int = 0x1234, fill: int = 0) -> np.ndarray:
    """A fragment frame: 20-byte IPv4 header (tot = 20 + payload, frag field) + payload."""
    h = np.zeros(20, np.uint8)
    h[0], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9] = (0x45, (20 + payload) >> 8, (20 + payload) & 0xFF,
                                                             ident >> 8, ident & 0xFF, frag >> 8, frag & 0xFF, 64, proto)
    h[12:20] = [10, 0, 0, 1, 10, 0, 0, 2]
    return np.concatenate([h, np.full(payload, fill, np.uint8)])


def run(frames, groups, cap=None):
    off = np.zeros(len(frames), np.uint64)
    pos = 0
    for i, f in enumerate(frames):
        off[i] = pos
        pos += f.size + 2
    buf = np.zeros(pos + 16, np.uint8)
    for i, f in enumerate(frames):
        buf[int(off[i]):int(off[i]) + f.size] = f
    d = G.ipv4_desc(off, np.array([f.size for f in frames], np.uint32))
    ng = len(groups)
    cap = cap or 70000
    od = G.ipv4_desc(np.arange(ng, dtype=np.uint64) * cap, np.full(ng, cap, np.uint32))
    out = np.zeros(ng * cap, np.uint8)
    ol, l4, v = O.ipv4_reassemble(buf, d, np.array(groups, np.uint32), out, od)
    return ol, l4, v, out


def test_reference_unit_cases():
    # check_complete case 1 / reassemble case 1: two 32-byte fragments, offsets 0 (MF) and 32
    ol, _, v, _ = run([frame(32, MF), frame(32, 32 >> 3)], [(0, 2)])
    assert ol[0] == 64 and v[0] == 1           # transport_receive called, 64 transport bytes
    # check_complete case 3: both carry MF -> not complete
    ol, _, v, _ = run([frame(32, MF), frame(32, (32 >> 3) | MF)], [(0, 2)])
    assert ol[0] == 0 and v[0] == 8
    # process_frag: a (0, MF), b (32, MF), c (64): buffer_len 96 + PICO_SIZE_IP4HDR
    ol, _, v, out = run([frame(32, MF, fill=1), frame(32, (32 >> 3) | MF, fill=2), frame(32, 64 >> 3, fill=3)],
                        [(0, 3)])
    assert ol[0] + 20 == 96 + 20 and v[0] == 1
    assert (out[20:52] == 1).all() and (out[52:84] == 2).all() and (out[84:116] == 3).all()


def test_order_duplicates_and_holes():
    # out of order arrival
    ol, _, v, out = run([frame(32, 64 >> 3, fill=3), frame(32, MF, fill=1), frame(32, (32 >> 3) | MF, fill=2)],
                        [(0, 3)])
    assert ol[0] == 96 and (out[20:52] == 1).all() and (out[84:116] == 3).all()
    # a repeated offset: the earlier arrival is kept (pico_tree_insert rejects the later)
    ol, _, v, out = run([frame(32, MF, fill=1), frame(32, MF, fill=9), frame(32, 32 >> 3, fill=2)], [(0, 3)])
    assert ol[0] == 64 and (out[20:52] == 1).all()
    # a hole: offsets 0, 64 -> incomplete
    ol, _, v, _ = run([frame(32, MF), frame(32, 64 >> 3)], [(0, 2)])
    assert v[0] == 8
    # overlap: offsets 0 (40 bytes), 32 -> bookmark 40 != 32 -> incomplete
    ol, _, v, _ = run([frame(40, MF), frame(32, 32 >> 3)], [(0, 2)])
    assert v[0] == 8
    # a fragment behind the completing one (reference UB: copy past the buffer) -> not reassembled
    ol, _, v, _ = run([frame(32, MF), frame(32, 32 >> 3), frame(32, 96 >> 3)], [(0, 3)])
    assert v[0] == 8


def py_reassemble(frames, proto):
    """Independent Python restatement of pico_fragments_check_complete + reassemble."""
    tree = {}
    for f in frames:
        fr = (int(f[6]) << 8) | int(f[7])
        o = (fr & 0x1FFF) << 3
        if o not in tree:
            tree[o] = f
    bm, parts, done = 0, [], False
    keys = sorted(tree)
    for i, o in enumerate(keys):
        f = tree[o]
        tl = ((int(f[2]) << 8) | int(f[3])) - 20
        if o != bm:
            return None
        bm += tl
        parts.append(f[20:20 + tl])
        if not ((int(f[6]) << 8 | int(f[7])) & MF):
            done = i == len(keys) - 1
            break
    if not done:
        return None
    t = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return t


@pytest.mark.parametrize("proto", [6, 17])
def test_seeded_sets_vs_python(proto):
    lens = [0, 7, 8, 100, 1480, 1481, 2960, 3001, 20000, 65515 - 1480 * 0]
    lens = [min(x, 65515) for x in lens]
    buf, off, flen, grp = synth.ipv4_fragments(lens, seed=9, proto=proto)
    d = G.ipv4_desc(off, flen)
    cap = np.array([(20 + x + 15) // 16 * 16 for x in lens], np.uint64)
    od = G.ipv4_desc(np.concatenate([[0], np.cumsum(cap)[:-1]]).astype(np.uint64), cap.astype(np.uint32))
    out = np.zeros(int(cap.sum()), np.uint8)
    ol, l4, v = O.ipv4_reassemble(buf, d, grp, out, od)
    for g, (first, cnt) in enumerate(grp.tolist()):
        frames = [buf[int(off[k]):int(off[k]) + int(flen[k])] for k in range(first, first + cnt)]
        t = py_reassemble(frames, proto)
        assert t is not None and ol[g] == t.size == lens[g]
        o = int(od["off"][g])
        np.testing.assert_array_equal(out[o + 20:o + 20 + t.size], t)
        if proto == 6 or (lens[g] >= 8 and (t[6] or t[7])):
            ph = np.concatenate([out[o + 12:o + 20], np.array([0, proto, t.size >> 8, t.size & 0xFF], np.uint8)])
            assert l4[g] == O.dualbuffer_checksum(ph, t)
        if lens[g] >= (20 if proto == 6 else 8):
            assert v[g] == 1 and l4[g] == 0            # synth writes a valid checksum
