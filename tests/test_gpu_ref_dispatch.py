"""The IPv6 RX transport dispatch on the GPU (IPv6 and Ethernet batches): the reference's byte-9
dispatch (the default, tests/test_ref_dispatch.py and tests/test_ref_rx.py pin it) and
PICO_CSUM_F_NXTHDR_DISPATCH, every wave shape vs the oracle on the IPv6 fixture, on random
datagrams whose header byte 9 selects TCP, UDP or nothing, and on a mixed Ethernet burst.
Run on an MI355X with `-m gpu`."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests import golden_data as G
from tests.test_gpu_fuzz import random_datagrams
from tests.test_gpu_parity import KERNELS, to_dev, u16, use_kernel

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0)


def _check(buf, desc, kernel, nx):
    wl, wv = O.batch_ipv6(buf, desc, nxthdr_dispatch=nx)
    use_kernel(kernel)
    l4, v = batch.ipv6_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), desc.size,
                                      flags=batch.F_NXTHDR_DISPATCH if nx else 0)
    np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"verdict kernel={kernel} nx={nx}")
    np.testing.assert_array_equal(u16(l4), wl, err_msg=f"l4 kernel={kernel} nx={nx}")


@pytest.mark.parametrize("kernel", list(KERNELS))
@pytest.mark.parametrize("nx", [False, True])
def test_dispatch_ipv6_fixture(kernel, nx):
    c = G.ipv6_cases()
    _check(c["buf"], G.ipv6_desc(c), kernel, nx)


@pytest.mark.parametrize("kernel", list(KERNELS))
@pytest.mark.parametrize("nx", [False, True])
def test_dispatch_random(kernel, nx):
    rng = np.random.default_rng(8100 + nx)
    n = 3000
    buf, desc = random_datagrams(rng, n, ipv6=True)
    offs = desc["off"].astype(np.int64)
    ok = offs + 10 <= buf.size
    buf[offs[ok] + 9] = rng.choice(np.array([6, 17, 6, 17, 0, 58], np.uint8), int(ok.sum()))
    _check(buf, desc, kernel, nx)


@pytest.mark.parametrize("kernel", ["auto", "fpw5", "fpw64"])
@pytest.mark.parametrize("nx", [False, True])
def test_dispatch_eth(kernel, nx):
    mac = bytes.fromhex("02005e0a0b0c")
    buf, off, flen, seeds, _ = synth.eth_batch(4000, seed=91, mac=mac)
    o = off.astype(np.int64)
    buf[o + 14 + 9] = np.random.default_rng(3).choice(np.array([6, 17, 1], np.uint8), o.size)
    desc = batch.make_desc(off, flen, seeds)
    wn, wl, wv = O.batch_eth(buf, desc, mac=mac, nxthdr_dispatch=nx)
    use_kernel(kernel)
    net, l4, v = batch.eth_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), desc.size,
                                          flags=batch.F_NXTHDR_DISPATCH if nx else 0, mac=mac)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(net), wn)
    np.testing.assert_array_equal(u16(l4), wl)
