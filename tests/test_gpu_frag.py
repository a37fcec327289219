"""GPU: IPv4 reassembly gather + transport check (pico_ipv4_reassemble_batch_dev) against the
oracle on seeded fragment sets -- out-of-order arrival, repeated offsets, holes, overlaps,
fragments behind the completing one, odd tails, UDP crc 0, TCP / UDP / other protocols,
64512-byte datagrams -- bit-exact on the outputs and on every reassembled byte."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests import golden_data as G
from tests.test_frag_oracle import MF, frame, run
from tests.test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu


def gpu_reassemble(buf, d, grp, od, out_size):
    out = torch.zeros(out_size, dtype=torch.uint8, device="cuda:0")
    ol, l4, v = batch.ipv4_reassemble_batch(to_dev(buf), to_dev(d.view(np.uint8)), d.size,
                                            to_dev(np.ascontiguousarray(grp, np.uint32).reshape(-1).view(np.int32)),
                                            out, to_dev(od.view(np.uint8)))
    torch.cuda.synchronize()
    return ol.cpu().numpy().view(np.uint32), l4.cpu().numpy().view(np.uint16), v.cpu().numpy(), out.cpu().numpy()


def check(buf, d, grp, od, out_size):
    out_o = np.zeros(out_size, np.uint8)
    wl, w4, wv = O.ipv4_reassemble(buf, d, grp, out_o, od)
    gl, g4, gv, out_g = gpu_reassemble(buf, d, grp, od, out_size)
    np.testing.assert_array_equal(gl, wl)
    np.testing.assert_array_equal(g4, w4)
    np.testing.assert_array_equal(gv, wv)
    for g in np.flatnonzero(wl):                        # every reassembled byte
        o, n = int(od["off"][g]), 20 + int(wl[g])
        np.testing.assert_array_equal(out_g[o:o + n], out_o[o:o + n], err_msg=f"datagram {g}")
    return wl, wv


def layout(lens, align=16, shift=0):
    cap = np.array([(20 + int(x) + align - 1) // align * align for x in lens], np.uint64) + np.uint64(align)
    off = np.concatenate([[0], np.cumsum(cap)[:-1]]).astype(np.uint64) + np.uint64(shift)
    return G.ipv4_desc(off, (cap - np.uint64(align)).astype(np.uint32)), int(cap.sum()) + shift + 16


@pytest.mark.parametrize("shift", [4, 12])
@pytest.mark.parametrize("proto", [6, 17, 1])
@pytest.mark.parametrize("payload", [1480, 8, 552, 64000])
def test_reassembly_vs_oracle(proto, payload, shift):
    rng = np.random.default_rng(proto * 100 + payload % 97)
    lens = rng.integers(0, 12000, 40).tolist() + [64512, 65515, 1, 7, 8, 9, 1480, 1481, 2959, 2960]
    if payload == 8:
        lens = [x for x in lens if x <= 4000]           # <= 512 fragments per datagram
    buf, off, flen, grp = synth.ipv4_fragments(lens, seed=proto + payload, proto=proto, frag_payload=payload)
    d = G.ipv4_desc(off, flen)
    od, size = layout(lens, shift=shift)              # 12: transports on 16-byte lines
    wl, wv = check(buf, d, grp, od, size)
    assert (wl == np.array(lens)).all()


def test_reassembly_edge_cases():
    sets = [
        ([frame(32, MF, fill=1), frame(32, 32 >> 3, fill=2)], "2 fragments (unit test case 1)"),
        ([frame(32, MF), frame(32, (32 >> 3) | MF)], "both MF: incomplete"),
        ([frame(32, 64 >> 3, fill=3), frame(32, MF, fill=1), frame(32, (32 >> 3) | MF, fill=2)], "out of order"),
        ([frame(32, MF, fill=1), frame(32, MF, fill=9), frame(32, 32 >> 3, fill=2)], "repeated offset"),
        ([frame(32, MF), frame(32, 64 >> 3)], "hole"),
        ([frame(40, MF), frame(32, 32 >> 3)], "overlap"),
        ([frame(32, MF), frame(32, 32 >> 3), frame(32, 96 >> 3)], "fragment behind the last"),
        ([frame(33, 0, proto=17, fill=5)], "single, odd, UDP crc != 0"),
        ([frame(48, MF, proto=6, fill=7), frame(31, 48 >> 3, proto=6, fill=8)], "TCP odd tail"),
        ([frame(16, MF, proto=17, fill=0), frame(16, 16 >> 3, proto=17, fill=4)], "UDP crc 0: not verified"),
    ]
    frames, grp = [], []
    for fs, _ in sets:
        grp.append((len(frames), len(fs)))
        frames.extend(fs)
    grp.append((0, 0))                                   # empty group
    grp.append((len(frames) - 1, 5))                     # past the descriptor array
    off = np.zeros(len(frames), np.uint64)
    pos = 3
    for i, f in enumerate(frames):
        off[i] = pos
        pos += f.size + 3                                # odd placement: unaligned payloads
    buf = np.zeros(pos + 16, np.uint8)
    for i, f in enumerate(frames):
        buf[int(off[i]):int(off[i]) + f.size] = f
    d = G.ipv4_desc(off, np.array([f.size for f in frames], np.uint32))
    od, size = layout([200] * len(grp))
    wl, wv = check(buf, d, np.array(grp, np.uint32), od, size)
    assert list(wv[:3]) == [1, 8, 1] and wv[-1] == 8 and wv[-2] == 8


def test_reassembly_limits():
    """Output region too small or misaligned, and a truncated fragment: not reassembled."""
    buf, off, flen, grp = synth.ipv4_fragments([3000, 3000, 3000], seed=4, proto=17)
    d = G.ipv4_desc(off, flen)
    od, size = layout([3000] * 3)
    od["len"][0] = 3000                                  # < 20 + 3000
    od["off"][1] += 2                                    # not 4-byte aligned
    d["len"][int(grp[2, 0])] -= 1                        # a payload past desc.len
    wl, wv = check(buf, d, grp, od, size)
    assert (wv == 8).all()
