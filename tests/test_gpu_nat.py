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
        batch.set_launch_override(0, 0, fpw)
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
