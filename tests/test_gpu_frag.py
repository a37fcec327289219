"""GPU: IPv4 / IPv6 reassembly gather + transport check (pico_ipv4_reassemble_batch_dev,
pico_ipv6_reassemble_batch_dev) against the oracle on seeded fragment sets -- out-of-order
arrival, repeated offsets, holes, overlaps, fragments behind the completing one, odd tails, UDP
crc 0, TCP / UDP / ICMP / other protocols, hop-by-hop headers before the fragment header, both
IPv6 dispatches, 64512-byte datagrams -- and against the reference-pinned fixture
(tests/golden/ref_reasm_cases.npz) -- bit-exact on the outputs and on every reassembled byte."""
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


@pytest.fixture(autouse=True, params=["auto", "flat"])
def reasm_path(request):
    """Every case through the launcher's own choice (the flat grid for batches of 512 datagrams
    or more, else one workgroup per datagram) and through the flat grid forced
    (pico_csum_set_reasm_flat(1))."""
    batch.set_reasm_flat(1 if request.param == "flat" else 0)
    yield request.param
    batch.set_reasm_flat(0)


def gpu_reassemble(buf, d, grp, od, out_size, v6=False, nx=False):
    out = torch.zeros(out_size, dtype=torch.uint8, device="cuda:0")
    args = (to_dev(buf), to_dev(d.view(np.uint8)), d.size,
            to_dev(np.ascontiguousarray(grp, np.uint32).reshape(-1).view(np.int32)), out, to_dev(od.view(np.uint8)))
    if v6:
        ol, l4, v = batch.ipv6_reassemble_batch(*args, flags=batch.F_NXTHDR_DISPATCH if nx else 0)
    else:
        ol, l4, v = batch.ipv4_reassemble_batch(*args)
    torch.cuda.synchronize()
    return ol.cpu().numpy().view(np.uint32), l4.cpu().numpy().view(np.uint16), v.cpu().numpy(), out.cpu().numpy()


def check(buf, d, grp, od, out_size, v6=False, nx=False):
    out_o = np.zeros(out_size, np.uint8)
    if v6:
        wl, w4, wv = O.ipv6_reassemble(buf, d, grp, out_o, od, nxthdr_dispatch=nx)
    else:
        wl, w4, wv = O.ipv4_reassemble(buf, d, grp, out_o, od)
    gl, g4, gv, out_g = gpu_reassemble(buf, d, grp, od, out_size, v6, nx)
    np.testing.assert_array_equal(gv, wv)
    np.testing.assert_array_equal(gl, wl)
    np.testing.assert_array_equal(g4, w4)
    H = 40 if v6 else 20
    for g in np.flatnonzero(wv != 8):                   # every reassembled byte
        o, n = int(od["off"][g]), H + int(wl[g])
        np.testing.assert_array_equal(out_g[o:o + n], out_o[o:o + n], err_msg=f"datagram {g}")
    return wl, wv


def layout(lens, align=16, shift=0, hdr=20):
    cap = np.array([(hdr + int(x) + align - 1) // align * align for x in lens], np.uint64) + np.uint64(align)
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


@pytest.mark.parametrize("shift", [8, 4])
@pytest.mark.parametrize("proto", [6, 17, 58])
@pytest.mark.parametrize("payload,hbh", [(1448, False), (8, False), (512, True), (64000, True)])
@pytest.mark.parametrize("nx", [False, True])
def test_ipv6_reassembly_vs_oracle(proto, payload, hbh, shift, nx):
    rng = np.random.default_rng(proto * 100 + payload % 97 + hbh)
    lens = (rng.integers(1, 1500, 30) * 8).tolist() + rng.integers(0, 9000, 10).tolist() + [
        65488, 65480, 65496, 1, 8, 9, 1448, 1449, 2896, 2904]
    if payload == 8:
        lens = [x for x in lens if x <= 4000]           # <= 512 fragments per datagram
    buf, off, flen, grp = synth.ipv6_fragments(lens, seed=proto + payload, proto=proto, frag_payload=payload,
                                               hbh=hbh, b9_proto=bool(rng.random() < 0.5))
    d = G.ipv4_desc(off, flen)
    od, size = layout(lens, shift=shift, hdr=40)          # 8: transports on 16-byte lines
    wl, wv = check(buf, d, grp, od, size, v6=True, nx=nx)
    assert (wv != 8).sum() >= len(lens) // 2


@pytest.mark.parametrize("fam,nx", [("v4", False), ("v6", False), ("v6", True)])
def test_reference_fixture(fam, nx):
    """The reference-pinned groups (make_ref_reasm.py): verdicts, lengths, transports, bytes."""
    c = G.ref_reasm_cases()
    p = fam + "_"
    d = G.ipv4_desc(c[p + "frag_off"], c[p + "frag_len"])
    od = G.ipv4_desc(c[p + "out_off"], c[p + "out_cap"])
    gl, g4, gv, out_g = gpu_reassemble(c[p + "buf"], d, c[p + "groups"], od, int(c[p + "out_size"][0]),
                                       fam == "v6", nx)
    np.testing.assert_array_equal(gv, c[p + ("verdict_nx" if nx else "verdict")])
    np.testing.assert_array_equal(gl, c[p + "len"])
    np.testing.assert_array_equal(g4, c[p + ("l4_nx" if nx else "l4")])
    H = 40 if fam == "v6" else 20
    for g in np.flatnonzero(gv != 8):
        o, n = int(c[p + "out_off"][g]), H + int(gl[g])
        np.testing.assert_array_equal(out_g[o:o + n], c[p + "exp_out"][o:o + n], err_msg=f"datagram {g}")


def test_ipv6_reassembly_limits():
    """Output region too small or misaligned, a truncated fragment, a datagram over 65535 bytes,
    and a fragment that does not walk to a fragment header: not reassembled."""
    buf, off, flen, grp = synth.ipv6_fragments([3000, 3000, 3000, 65496, 3000], seed=5, proto=17)
    d = G.ipv4_desc(off, flen)
    od, size = layout([3000, 3000, 3000, 65496, 3000], hdr=40)
    od["len"][0] = 3000                                  # < 40 + 3000
    od["off"][1] += 2                                    # not 4-byte aligned
    d["len"][int(grp[2, 0])] -= 1                        # a payload past desc.len
    f4 = int(off[int(grp[4, 0])])
    buf[f4 + 6] = 17                                     # no fragment header: UDP straight away
    wl, wv = check(buf, d, grp, od, size, v6=True)
    assert (wv == 8).all()


@pytest.mark.parametrize("v6", [False, True])
@pytest.mark.parametrize("n", [1600, 3200])
def test_batch_shapes(n, v6, reasm_path):
    """Batches below and above the launcher's switch to one wave per datagram (3072) -- both on
    the flat grid (>= 512 datagrams) unless forced off -- with datagrams of more than 64 fragments
    per wave (the gather's metadata blocks; the flat grid's SLOW plans)."""
    rng = np.random.default_rng(n + v6)
    lens = rng.integers(0, 3000, n)
    lens[rng.integers(0, n, 24)] = rng.integers(8200, 9000, 24)   # 129-141 fragments of 64 B
    lens = lens.tolist()
    if v6:
        buf, off, flen, grp = synth.ipv6_fragments(lens, seed=n, proto=6, frag_payload=64)
    else:
        buf, off, flen, grp = synth.ipv4_fragments(lens, seed=n, proto=6, frag_payload=64)
    d = G.ipv4_desc(off, flen)
    od, size = layout(lens, shift=4, hdr=40 if v6 else 20)
    wl, wv = check(buf, d, grp, od, size, v6=v6)
    assert (wv != 8).all() and (wl == np.array(lens)).all()
    if reasm_path == "auto":                             # and one workgroup per datagram
        batch.set_reasm_flat(2)
        wl, wv = check(buf, d, grp, od, size, v6=v6)
        assert (wv != 8).all() and (wl == np.array(lens)).all()


@pytest.mark.parametrize("v6", [False, True])
@pytest.mark.parametrize("shift", [0, 4, 8, 12])
@pytest.mark.parametrize("payload", [8, 16, 24, 40])
def test_unit_grid(payload, shift, v6):
    """The gather's units follow the output's 16-byte lines: every placement of the transport
    in its line (o = 0, 4, 8, 12 via the region shift and the 8-byte fragment offsets), fragments
    shorter than a unit (first unit = last unit, o + len < 16), odd and 1-3-byte tails, shuffled
    arrival -- every reassembled byte and checksum against the oracle."""
    rng = np.random.default_rng(payload * 16 + shift + v6)
    lens = list(range(0, 70)) + rng.integers(70, 700, 30).tolist()
    if v6:
        buf, off, flen, grp = synth.ipv6_fragments(lens, seed=payload + shift, proto=17, frag_payload=payload)
    else:
        buf, off, flen, grp = synth.ipv4_fragments(lens, seed=payload + shift, proto=6, frag_payload=payload)
    d = G.ipv4_desc(off, flen)
    od, size = layout(lens, shift=shift, hdr=40 if v6 else 20)
    wl, wv = check(buf, d, grp, od, size, v6=v6)
    ok = wv != 8
    assert ok.mean() > 0.9 and (wl[ok] == np.array(lens)[ok]).all()


def _flat_case(n, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 6000, n).tolist()
    buf, off, flen, grp = synth.ipv4_fragments(lens, seed=seed, proto=6, frag_payload=552)
    d = G.ipv4_desc(off, flen)
    od, size = layout(lens, shift=4)
    out_o = np.zeros(size, np.uint8)
    want = O.ipv4_reassemble(buf, d, grp, out_o, od)
    dev = (to_dev(buf), to_dev(d.view(np.uint8)), d.size,
           to_dev(np.ascontiguousarray(grp, np.uint32).reshape(-1).view(np.int32)), to_dev(od.view(np.uint8)))
    return dev, od, size, want, out_o


def _check_flat(res, out, od, want, out_o):
    ol, l4, v = (x.cpu().numpy() for x in res)
    np.testing.assert_array_equal(v, want[2])
    np.testing.assert_array_equal(ol.view(np.uint32), want[0])
    np.testing.assert_array_equal(l4.view(np.uint16), want[1])
    o_g = out.cpu().numpy()
    for g in np.flatnonzero(want[2] != 8):
        o, n = int(od["off"][g]), 20 + int(want[0][g])
        np.testing.assert_array_equal(o_g[o:o + n], out_o[o:o + n], err_msg=f"datagram {g}")


def test_flat_grid_graph_capture():
    """The flat grid captured into a graph (its scratch then owned by the graph): replays match the
    oracle, and eager calls afterwards too (after the graph is destroyed as well)."""
    (b, d, nf, grp, od_d), od, size, want, out_o = _flat_case(1500, 71)
    outs = [torch.zeros(size, dtype=torch.uint8, device="cuda:0") for _ in range(2)]
    res = [batch.ipv4_reassemble_batch(b, d, nf, grp, o, od_d) for o in outs]   # warm (eager)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for o, r in zip(outs, res):
                batch.ipv4_reassemble_batch(b, d, nf, grp, o, od_d, stream=s, results=r)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        for o, r in zip(outs, res):
            o.zero_()
            for x in r:
                x.zero_()
        g.replay()
        torch.cuda.synchronize()
        for o, r in zip(outs, res):
            _check_flat(r, o, od, want, out_o)
    o = torch.zeros(size, dtype=torch.uint8, device="cuda:0")
    r = batch.ipv4_reassemble_batch(b, d, nf, grp, o, od_d, stream=s)
    torch.cuda.synchronize()
    _check_flat(r, o, od, want, out_o)
    del g                                                # the graph's scratch freed by the next call
    torch.cuda.synchronize()
    o.zero_()
    r = batch.ipv4_reassemble_batch(b, d, nf, grp, o, od_d)
    torch.cuda.synchronize()
    _check_flat(r, o, od, want, out_o)


def test_flat_grid_streams_and_sizes():
    """Calls alternating between two streams (each its own scratch), a larger batch after a smaller
    one on the same stream (the scratch grows), then the smaller again -- all against the oracle."""
    small = _flat_case(1100, 73)
    large = _flat_case(3000, 74)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    runs = []
    for case, st in ((small, s1), (small, s2), (large, s1), (large, s2), (small, s1)):
        (b, d, nf, grp, od_d), od, size, want, out_o = case
        o = torch.zeros(size, dtype=torch.uint8, device="cuda:0")
        st.wait_stream(torch.cuda.current_stream())
        r = batch.ipv4_reassemble_batch(b, d, nf, grp, o, od_d, stream=st)
        runs.append((r, o, case))
    torch.cuda.synchronize()
    for r, o, (_, od, size, want, out_o) in runs:
        _check_flat(r, o, od, want, out_o)


def _with_retransmits(buf, off, flen, grp, seed, per=(1, 3), same=0.0, hdr=20):
    """Every datagram gets per[0]..per[1] retransmitted fragments: a copy of one of its fragments
    at a random place in its arrival order -- before the original (the copy is then the kept one)
    or after it (rejected by pico_tree_insert).  A copy carries the original's bytes with
    probability `same` (a true retransmission), else different payload bytes (behind `hdr`)."""
    rng = np.random.default_rng(seed)
    extra, new_off, new_len, new_grp = [], [], [], []
    pos = buf.size
    for first, cnt in grp:
        orig = [(int(off[first + k]), int(flen[first + k])) for k in range(cnt)]
        order = list(orig)
        for _ in range(int(rng.integers(per[0], per[1] + 1)) if cnt else 0):
            o, n = orig[int(rng.integers(0, cnt))]
            f = buf[o:o + n].copy()
            if rng.random() >= same:
                f[hdr:] = rng.integers(0, 256, n - hdr, dtype=np.uint8)
            extra.append(f)
            order.insert(int(rng.integers(0, len(order) + 1)), (pos, n))
            pos += n
        new_grp.append((len(new_off), len(order)))
        new_off += [o for o, _ in order]
        new_len += [n for _, n in order]
    nb = np.concatenate([buf] + extra + [np.zeros(16, np.uint8)])
    return nb, np.array(new_off, np.uint64), np.array(new_len, np.uint32), np.array(new_grp, np.uint32)


@pytest.mark.parametrize("payload", [1480, 552])
def test_flat_grid_retransmits(payload):
    """A batch of 700 datagrams (the flat grid under both fixture settings), every one with 1-3
    retransmitted fragments carrying different payload bytes, arrival shuffled: the earliest
    arrival of each offset is kept, as the reference's fragment tree does, on every datagram."""
    rng = np.random.default_rng(payload)
    lens = rng.integers(1, 20000, 700).tolist()
    buf, off, flen, grp = synth.ipv4_fragments(lens, seed=payload, proto=6, frag_payload=payload)
    buf, off, flen, grp = _with_retransmits(buf, off, flen, grp, seed=payload + 1)
    d = G.ipv4_desc(off, flen)
    od, size = layout(lens, shift=4)
    wl, wv = check(buf, d, grp, od, size)
    assert (wv != 8).mean() > 0.9


@pytest.mark.parametrize("v6", [False, True])
@pytest.mark.parametrize("same", [1.0, 0.7])
def test_flat_grid_true_retransmits(v6, same):
    """Retransmissions carrying the original's bytes (all of them, or 70 % mixed with altered
    copies) on 800 datagrams: the flat grid's planner keeps such a plan GOOD and subtracts the
    copy's sum; an altered copy sends its datagram to the finish's workgroup path.  Every
    verdict, checksum and reassembled byte against the oracle (both fixture settings)."""
    rng = np.random.default_rng(17 + v6)
    lens = rng.integers(1, 24000, 800).tolist()
    if v6:
        lens = [x // 8 * 8 + 8 for x in lens]
        buf, off, flen, grp = synth.ipv6_fragments(lens, seed=31, proto=6, frag_payload=1448)
    else:
        buf, off, flen, grp = synth.ipv4_fragments(lens, seed=31, proto=6, frag_payload=1480)
    buf, off, flen, grp = _with_retransmits(buf, off, flen, grp, seed=32 + v6, per=(0, 2), same=same,
                                            hdr=48 if v6 else 20)
    d = G.ipv4_desc(off, flen)
    od, size = layout(lens, shift=8 if v6 else 4, hdr=40 if v6 else 20)
    wl, wv = check(buf, d, grp, od, size, v6=v6)
    ok = wv != 8
    assert ok.mean() > 0.9
    if same == 1.0:
        assert (wv == 1).mean() > 0.99                   # the kept bytes are the originals: valid TCP


@pytest.mark.parametrize("v6", [False, True])
def test_flat_grid_two_fragments_a_lane(v6, reasm_path):
    """Datagrams of 65-128 fragments (64 KiB over 552 / 520-byte fragments: the planner holds two
    fragments a lane; the launcher's automatic choice is the flat grid up to 128 a datagram on
    average), some with retransmitted fragments -- the same bytes or altered, in either half of the
    arrival order -- on 600 datagrams: every verdict, checksum and reassembled byte against the
    oracle, and again on one workgroup per datagram.  (More than 128 fragments: test_batch_shapes.)"""
    rng = np.random.default_rng(23 + v6)
    pl = 520 if v6 else 552
    lens = rng.integers(34000, 65000, 600)
    lens[rng.integers(0, 600, 20)] = rng.integers(0, 3000, 20)            # and a few short ones
    lens = [int(x) // 8 * 8 + 8 if v6 else int(x) for x in lens]
    if v6:
        buf, off, flen, grp = synth.ipv6_fragments(lens, seed=41, proto=6, frag_payload=pl)
    else:
        buf, off, flen, grp = synth.ipv4_fragments(lens, seed=41, proto=6, frag_payload=pl)
    buf, off, flen, grp = _with_retransmits(buf, off, flen, grp, seed=42 + v6, per=(0, 3), same=0.6,
                                            hdr=48 if v6 else 20)
    assert ((grp[:, 1] > 64) & (grp[:, 1] <= 128)).mean() > 0.8
    d = G.ipv4_desc(off, flen)
    od, size = layout(lens, shift=8 if v6 else 4, hdr=40 if v6 else 20)
    wl, wv = check(buf, d, grp, od, size, v6=v6)
    assert (wv != 8).mean() > 0.9
    if reasm_path == "auto":                             # and one workgroup per datagram
        batch.set_reasm_flat(2)
        wl2, wv2 = check(buf, d, grp, od, size, v6=v6)
        assert (wv2 == wv).all() and (wl2 == wl).all()
