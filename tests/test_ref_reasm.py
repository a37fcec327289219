"""The reassembly restatement (oracle_ipv4_reassemble / oracle_ipv6_reassemble) against the
reference's own compiled fragment path (CPU).

tests/golden/ref_reasm_cases.npz (made by tests/golden/make_ref_reasm.py) holds 300 IPv4 and 300
IPv6 fragment groups -- shuffled arrival, holes, repeats, flipped payload bits, hop-by-hop headers
before the fragment header, ND / MLD ICMPv6 types, byte-9 dispatch -- with the datagram
pico_fragments.c hands to the transport (bytes, length) and pico_transport_crc_check's verdict
on it, from the reference compiled unmodified (oracle/_ref/libref_rx.so).  When that library is
present, a sample of the groups is also re-run live."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_data as G
from tests.test_ref_rx import REF_RX


def _run(c, fam, nx=False):
    p = fam + "_"
    d = np.zeros(c[p + "frag_off"].size, O.DESC_DTYPE)
    d["off"], d["len"] = c[p + "frag_off"], c[p + "frag_len"]
    od = np.zeros(c[p + "out_off"].size, O.DESC_DTYPE)
    od["off"], od["len"] = c[p + "out_off"], c[p + "out_cap"]
    out = np.zeros(int(c[p + "out_size"][0]), np.uint8)
    if fam == "v6":
        r = O.ipv6_reassemble(c[p + "buf"], d, c[p + "groups"], out, od, nxthdr_dispatch=nx)
    else:
        r = O.ipv4_reassemble(c[p + "buf"], d, c[p + "groups"], out, od)
    return r + (out,)


@pytest.mark.parametrize("fam", ["v4", "v6"])
def test_oracle_matches_reference_fixture(fam):
    c = G.ref_reasm_cases()
    p = fam + "_"
    ol, l4, v, out = _run(c, fam)
    np.testing.assert_array_equal(v, c[p + "verdict"])
    np.testing.assert_array_equal(ol, c[p + "len"])
    np.testing.assert_array_equal(l4, c[p + "l4"])
    H = 40 if fam == "v6" else 20
    for g in np.flatnonzero(v != 8):
        o = int(c[p + "out_off"][g])
        np.testing.assert_array_equal(out[o:o + H + ol[g]], c[p + "exp_out"][o:o + H + ol[g]])
    assert c[p + "pinned_bytes"].all() and c[p + "pinned_verdict"].mean() > 0.6
    assert set(np.unique(v).tolist()) == {1, 4, 8}
    if fam == "v6":
        _, l4nx, vnx, _ = _run(c, fam, nx=True)
        np.testing.assert_array_equal(vnx, c["v6_verdict_nx"])
        np.testing.assert_array_equal(l4nx, c["v6_l4_nx"])
        assert (vnx != v).any()                        # the byte-9 dispatch matters on these groups


@pytest.mark.skipif(not os.path.exists(REF_RX), reason="oracle/_ref/libref_rx.so not built (make -C oracle refrx)")
@pytest.mark.parametrize("fam", ["v4", "v6"])
def test_reference_rerun_live(fam):
    """The compiled reference again, on every 5th group (catches a stale fixture)."""
    R = ctypes.CDLL(REF_RX)
    R.rr_ipv4_link.argtypes = [ctypes.c_uint32]
    R.rr_reasm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    assert R.rr_init() == 0
    c = G.ref_reasm_cases()
    p = fam + "_"
    v6 = fam == "v6"
    H = 40 if v6 else 20
    buf = c[p + "buf"]
    for g, (first, cnt) in list(enumerate(c[p + "groups"].tolist()))[::5]:
        offs = np.ascontiguousarray(c[p + "frag_off"][first:first + cnt])
        lens = np.ascontiguousarray(c[p + "frag_len"][first:first + cnt])
        if not v6 and cnt:
            o = int(offs[0])
            R.rr_ipv4_link(int.from_bytes(bytes(buf[o + 16:o + 20]), "little"))
        rout = np.zeros(70000, np.uint8)
        rl, rm, rc = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_int(0)
        ok = R.rr_reasm(int(v6), buf.ctypes.data, offs.ctypes.data if cnt else None,
                        lens.ctypes.data if cnt else None, cnt, rout.ctypes.data, 70000,
                        ctypes.byref(rl), ctypes.byref(rm), ctypes.byref(rc))
        want_v = int(c[p + "verdict"][g])
        if not ok:
            assert want_v == 8
            continue
        o = int(c[p + "out_off"][g])
        assert rl.value == c[p + "len"][g]
        np.testing.assert_array_equal(rout[:H + rl.value], c[p + "exp_out"][o:o + H + rl.value])
        if rm.value in (6, 17) and rc.value >= 0:
            assert want_v == (1 if rc.value else 4)


@pytest.mark.skipif(not O.ref_reasm_available(), reason="oracle/_ref/libref_rx_O3.so not built (needs /root/reference)")
@pytest.mark.parametrize("v6", [False, True])
def test_reference_batch_baseline(v6, capfd):
    """bench.py's reassembly CPU baseline: the -O3 reference stack's rr_reasm_batch reassembles
    and transport-checks every datagram of a synthetic batch (IPv4 header checksums filled in, as
    the baseline does), the oracle agreeing, and none of the stack's debug output reaches
    stdout."""
    from picotcp_amd import synth
    lens = [64512, 3000, 2961, 20000] * 4              # (fragmented: bench.py's batches are)
    if v6:
        buf, off, flen, grp = synth.ipv6_fragments(lens, seed=9, proto=6, frag_payload=1448)
    else:
        buf, off, flen, grp = synth.ipv4_fragments(lens, seed=9, proto=6, frag_payload=1480)
        O.fix_ipv4_header_crcs(buf, off)
    d = np.zeros(off.size, O.DESC_DTYPE)
    d["off"], d["len"] = off, flen
    od = np.zeros(len(lens), O.DESC_DTYPE)
    H = 40 if v6 else 20
    od["off"] = np.arange(len(lens), dtype=np.uint64) * 65600
    od["len"] = 65600
    out = np.zeros(65600 * len(lens), np.uint8)
    wl, w4, wv = (O.ipv6_reassemble if v6 else O.ipv4_reassemble)(buf, d, grp, out, od)
    o0 = int(off[0])
    O.ref_reasm_link(v6, bytes(buf[o0 + 24:o0 + 40]) if v6 else bytes(buf[o0 + 16:o0 + 20]))
    secs, done, chk = O.ref_reasm_batch(v6, buf, off, flen, grp)
    assert done == len(lens) and (wv != 8).all()
    assert chk == int((wv == 1).sum()) == len(lens)
    assert secs > 0
    assert capfd.readouterr().out == ""
