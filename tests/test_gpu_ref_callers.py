"""GPU: the fused IPv4 / IPv6 kernels and the seeded raw batch against the values the
reference's OWN compiled callers return (tests/golden/ref_callers.npz, from
pico_tcp_checksum_ipv4/_ipv6, pico_udp_checksum_ipv4/_ipv6, pico_icmp6_checksum and
pico_mld_checksum; tests/golden/make_ref_callers.py), bit-exact, on every descriptor
kernel variant."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from picotcp_amd import _lib, batch
from tests import golden_data as G
from tests.test_gpu_parity import KERNELS, to_dev, u16, use_kernel

pytestmark = pytest.mark.gpu

VARIANTS = list(KERNELS)


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0)


@pytest.mark.parametrize("kernel", VARIANTS)
@pytest.mark.parametrize("tx", [False, True])
def test_ipv4_transport_vs_reference_callers(kernel, tx):
    rc, c = G.ref_callers(), G.ipv4_cases()
    ref = rc["v4_tx" if tx else "v4_rx"]
    use_kernel(kernel)
    buf = to_dev(c["tx_buf" if tx else "buf"])
    d = to_dev(G.ipv4_desc(c["net"], c["avail"]).view(np.uint8))
    _, l4, _ = batch.ipv4_checksum_batch(buf, d, c["net"].size, flags=_lib.F_TX if tx else 0)
    got = u16(l4).astype(np.int32)
    m = ref >= 0
    np.testing.assert_array_equal(got[m], ref[m])


@pytest.mark.parametrize("kernel", VARIANTS)
@pytest.mark.parametrize("tx", [False, True])
def test_ipv6_transport_vs_reference_callers(kernel, tx):
    rc, c = G.ref_callers(), G.ipv6_cases()
    ref = rc["v6_tx" if tx else "v6_rx"]
    use_kernel(kernel)
    buf = to_dev(c["tx_buf" if tx else "buf"])
    d = to_dev(G.ipv6_desc(c).view(np.uint8))
    l4, _ = batch.ipv6_checksum_batch(buf, d, c["net"].size, flags=_lib.F_TX if tx else 0)
    got = u16(l4).astype(np.int32)
    m = ref >= 0
    np.testing.assert_array_equal(got[m], ref[m])


@pytest.mark.parametrize("kernel", VARIANTS)
def test_ipv6_nxthdr_dispatch_vs_reference_callers(kernel):
    """F_NXTHDR_DISPATCH: the transport's own protocol picks the caller."""
    rc, c = G.ref_callers(), G.ipv6_cases()
    ref = rc["v6_rx_nx"]
    use_kernel(kernel)
    d = to_dev(G.ipv6_desc(c).view(np.uint8))
    l4, _ = batch.ipv6_checksum_batch(to_dev(c["buf"]), d, c["net"].size, flags=_lib.F_NXTHDR_DISPATCH)
    got = u16(l4).astype(np.int32)
    m = ref >= 0
    np.testing.assert_array_equal(got[m], ref[m])


@pytest.mark.parametrize("kernel", list(KERNELS))
@pytest.mark.parametrize("tx", [False, True])
def test_mld_checksum_vs_reference(kernel, tx):
    """pico_mld_checksum (pico_mld.c:421-437) as a raw batch: region = the report behind the
    8-byte router alert, seed = pico_ipv6_pseudo_partial(src, dst, 58, len - 8); TX reads the
    report's crc (region offset 2) as zero and writes it in place."""
    rc = G.ref_callers()
    lib = _lib.load()
    buf = rc["mld_buf"]
    n = rc["mld_net"].size
    desc = np.zeros(n, dtype=batch.DESC_DTYPE)
    for i, (o, size) in enumerate(zip(rc["mld_net"].astype(int), rc["mld_size"].astype(int))):
        h = np.ascontiguousarray(buf[o:o + 40])
        desc["off"][i] = o + 48
        desc["len"][i] = size - 48
        desc["seed"][i] = lib.pico_ipv6_pseudo_partial(h[8:24].ctypes.data, h[24:40].ctypes.data, 58, size - 48)
    use_kernel(kernel)
    dbuf = to_dev(buf)
    out = batch.checksum_batch(dbuf, to_dev(desc.view(np.uint8)), n, crc_off=2 if tx else -1,
                               flags=_lib.F_WRITE if tx else 0)
    ref = rc["mld_tx" if tx else "mld_rx"]
    np.testing.assert_array_equal(u16(out).astype(np.int32), ref)
    if tx:                     # the stored field is short_be(ret): the report now verifies to 0
        back = dbuf.cpu().numpy()
        for i, o in enumerate(desc["off"].astype(int)):
            assert (int(back[o + 2]) << 8 | int(back[o + 3])) == ref[i]
    torch.cuda.synchronize()
