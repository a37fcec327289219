"""The NAT restatement (oracle_batch_ipv4_nat) against the reference's own compiled
pico_ipv4_nat_outbound / pico_ipv4_nat_inbound (modules/pico_nat.c:424-545), CPU.

tests/golden/ref_nat_cases.npz (made by tests/golden/make_ref_nat.py) holds 1310 datagrams:
TCP / UDP / ICMPv4 / GRE outbound from private hosts (options, valid / corrupted / zero transport
checksums) and inbound replies on the outbound tuples' ports or on ports no tuple holds, with the
reference's bytes after the call and its return value; plus fragments, infeasible lengths and
short transports the stack never hands to NAT (restatement only: "parity unpinned" for those).
When oracle/_ref/libref_rx.so is present, fresh datagrams are also run through the reference
live (a private copy of the library) and compared with the restatement on the reference's own
NAT ports."""
from __future__ import annotations

import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_data as G
from tests.golden import make_ref_nat as M


def cases():
    z = np.load(os.path.join(G.GOLDEN, "ref_nat_cases.npz"))
    c = {k: z[k] for k in z.files}
    c["nat"] = c["nat"].view(O.NAT_DTYPE)
    d = np.zeros(c["off"].size, O.DESC_DTYPE)
    d["off"], d["len"] = c["off"], c["avail"]
    c["desc"] = d
    return c


def test_oracle_matches_reference_fixture():
    c = cases()
    got = c["buf"].copy()
    on, ol, v = O.batch_ipv4_nat(got, c["desc"], c["nat"])
    np.testing.assert_array_equal(got, c["want"])                 # every byte the reference wrote
    np.testing.assert_array_equal(v, c["verdict"])
    called = c["ret"] != -9
    assert (v[called & (c["ret"] == 0)] == 1).all() and (v[called & (c["ret"] == -1)] == 32).all()
    # the values reported are the ones stored: header crc at +10, transport crc at +16 / +6
    for i in np.flatnonzero(v == 1)[:200]:
        o = int(c["off"][i])
        h = c["want"][o:o + 60]
        assert on[i] == (int(h[10]) << 8 | int(h[11]))
        hl = 4 * (int(h[0]) & 15)
        if h[9] in (6, 17):
            x = o + hl + (16 if h[9] == 6 else 6)
            assert ol[i] == (int(c["want"][x]) << 8 | int(c["want"][x + 1]))
    # corrupted and zero UDP checksums come out recomputed, as the reference does
    assert (c["ret"] == 0).sum() > 900 and set(np.unique(v).tolist()) == {1, 8, 16, 32}


@pytest.mark.skipif(not os.path.exists(M.REF_RX), reason="oracle/_ref/libref_rx.so not built (make -C oracle refrx)")
def test_reference_rerun_live():
    """Fresh outbound datagrams through the reference now; the restatement, given the NAT ports the
    reference chose, writes the same bytes."""
    R = M.ref_lib()
    rng = np.random.default_rng(77)
    nat_addr = int.from_bytes(M.NAT_ADDR, "little")
    for k in range(120):
        proto = [6, 17, 17, 1][k % 4]
        tl = int(rng.integers(20 if proto == 6 else 8, 400))
        d = M.datagram(rng, proto, tl, bytes([10, 1, 2, 3 + k % 50]), bytes([203, 0, 113, 5]), 2000 + k, 443,
                       opts=k % 3, l4=["valid", "bad", "zero"][k % 3] if proto == 17 else "bad")
        ref = d.copy()
        assert R.rr_nat(1, ref.ctypes.data, ref.size, nat_addr) == 0
        hl = 4 * (int(d[0]) & 15)
        rec = np.zeros(1, O.NAT_DTYPE)
        rec["dir"] = 1
        if proto != 1:
            rec["addr"] = int.from_bytes(bytes(ref[12:16]), "little")
            rec["port"] = int.from_bytes(bytes(ref[hl:hl + 2]), "little")
        got = d.copy()
        desc = np.zeros(1, O.DESC_DTYPE)
        desc["len"] = d.size
        on, ol, v = O.batch_ipv4_nat(got, desc, rec)
        assert v[0] == 1
        np.testing.assert_array_equal(got, ref, err_msg=f"case {k} proto {proto}")
