"""GPU: the fused IPv4 (MODE 1) and IPv6 (MODE 2) descriptor kernels directly on the reference's
own RX verdicts, tests/golden/ref_rx_cases.npz (tests/golden/make_ref_rx.py: 5000 IPv4 + 5000
IPv6 datagrams through pico_ipv4_process_in / pico_ipv6_extension_headers /
pico_transport_crc_check compiled unmodified from /root/reference).

Every kernel variant sees the fixture:
  * layouts -- the fixture's own (datagrams a few bytes apart: stream-order waves, K4s), repacked
    back to back with odd gaps (K4s, odd starts), and spread one per 4 KiB slot at a random line
    offset (no wave is one dense span: the sorted rounds, K4);
  * frames per wave -- automatic, 1, 5 and 64 (launch override group 2).
Pinned rows must equal the reference's verdict and checksums; every row (pinned or restatement-
only) must equal the oracle's."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch
from tests import golden_data as G
from tests.test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0)


def relayout(buf, off, avail, how, seed):
    """The same datagram bytes at new offsets: 'fixture' (as recorded), 'packed' (back to back,
    0-3 byte gaps) or 'sparse' (one per 4 KiB slot, 0-15 bytes into it)."""
    if how == "fixture":
        return buf, off
    rng = np.random.default_rng(seed)
    n = off.size
    if how == "packed":
        gaps = rng.integers(0, 4, n)
        new = np.cumsum(np.concatenate([[0], avail[:-1].astype(np.int64) + gaps[1:]])) + gaps[0]
    else:
        new = np.arange(n, dtype=np.int64) * 4096 + rng.integers(0, 16, n)
    nb = np.zeros(int(new[-1]) + int(avail[-1]) + 64, np.uint8)
    for o, a, q in zip(off.astype(np.int64), avail.astype(np.int64), new):
        nb[q:q + a] = buf[o:o + a]
    return nb, new.astype(np.uint64)


@pytest.mark.parametrize("how", ["fixture", "packed", "sparse"])
@pytest.mark.parametrize("fpw", [0, 1, 5, 64])
def test_ipv4_kernel_on_reference_verdicts(how, fpw):
    c = G.ref_rx_cases()
    buf, off = relayout(c["v4_buf"], c["v4_off"], c["v4_avail"], how, 3)
    desc = batch.make_desc(off, c["v4_avail"])
    if fpw:
        batch.set_launch_override(2, fpw=fpw)
    on, ol, v = batch.ipv4_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), desc.size)
    torch.cuda.synchronize()
    on, ol, v = on.cpu().numpy().view(np.uint16), ol.cpu().numpy().view(np.uint16), v.cpu().numpy()
    pin = c["v4_pinned"]
    np.testing.assert_array_equal(v[pin], c["v4_verdict"][pin])
    np.testing.assert_array_equal(on[pin], c["v4_net"][pin])
    np.testing.assert_array_equal(ol[pin], c["v4_l4"][pin])
    wn, wl, wv = O.batch_ipv4(buf, desc)
    np.testing.assert_array_equal(v, wv)
    np.testing.assert_array_equal(on, wn)
    np.testing.assert_array_equal(ol, wl)


@pytest.mark.parametrize("how", ["fixture", "packed", "sparse"])
@pytest.mark.parametrize("fpw", [0, 1, 5, 64])
def test_ipv6_kernel_on_reference_verdicts(how, fpw):
    c = G.ref_rx_cases()
    buf, off = relayout(c["v6_buf"], c["v6_off"], c["v6_avail"], how, 4)
    desc = batch.make_desc(off, c["v6_avail"])          # seed 0: the kernel walks the extension headers
    if fpw:
        batch.set_launch_override(2, fpw=fpw)
    l4, v = batch.ipv6_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), desc.size)
    torch.cuda.synchronize()
    l4, v = l4.cpu().numpy().view(np.uint16), v.cpu().numpy()
    pin = c["v6_pinned"]
    np.testing.assert_array_equal(v[pin], c["v6_verdict"][pin])
    np.testing.assert_array_equal(l4[pin], c["v6_l4"][pin])
    wl, wv = O.batch_ipv6(buf, desc)
    np.testing.assert_array_equal(v, wv)
    np.testing.assert_array_equal(l4, wl)
