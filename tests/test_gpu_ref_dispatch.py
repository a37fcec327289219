"""PICO_CSUM_F_REF_DISPATCH on the GPU (IPv6 and Ethernet batches, RX): every sorted-kernel
variant vs the oracle (tests/test_ref_dispatch.py pins its semantics) on the IPv6 fixture, on
random datagrams whose header byte 9 selects TCP, UDP or nothing, and on a mixed Ethernet
burst.  Run on an MI355X with `-m gpu`."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests import golden_data as G
from tests.test_gpu_fuzz import random_datagrams
from tests.test_gpu_parity import KERNELS, to_dev, u16, use_kernel
from tests.test_gpu_stream import dense_datagrams

pytestmark = pytest.mark.gpu
SORTED = ["auto"] + [k for k, v in KERNELS.items() if v is not None and v[0] == 2] + ["flat"]


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0)


def _check(buf, desc, kernel):
    wl, wv = O.batch_ipv6(buf, desc, ref_dispatch=True)
    use_kernel(kernel)           # "flat": the host routes the flag to the sorted kernel anyway
    l4, v = batch.ipv6_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), desc.size,
                                      flags=batch.F_REF_DISPATCH)
    np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"verdict kernel={kernel}")
    np.testing.assert_array_equal(u16(l4), wl, err_msg=f"l4 kernel={kernel}")


@pytest.mark.parametrize("kernel", SORTED)
def test_ref_dispatch_ipv6_fixture(kernel):
    c = G.ipv6_cases()
    _check(c["buf"], G.ipv6_desc(c), kernel)


@pytest.mark.parametrize("kernel", SORTED)
@pytest.mark.parametrize("dense", [False, True])
def test_ref_dispatch_random(kernel, dense):
    rng = np.random.default_rng(8100 + dense)
    n = 3000
    buf, desc = dense_datagrams(rng, n, ipv6=True, breaks=False) if dense else random_datagrams(rng, n, ipv6=True)
    offs = desc["off"].astype(np.int64)
    ok = offs + 10 <= buf.size
    buf[offs[ok] + 9] = rng.choice(np.array([6, 17, 6, 17, 0, 58], np.uint8), int(ok.sum()))
    _check(buf, desc, kernel)


@pytest.mark.parametrize("kernel", SORTED[:4])
def test_ref_dispatch_eth(kernel):
    mac = bytes.fromhex("02005e0a0b0c")
    buf, off, flen, seeds, _ = synth.eth_batch(4000, seed=91, mac=mac)
    o = off.astype(np.int64)
    buf[o + 14 + 9] = np.random.default_rng(3).choice(np.array([6, 17, 1], np.uint8), o.size)
    desc = batch.make_desc(off, flen, seeds)
    wn, wl, wv = O.batch_eth(buf, desc, mac=mac, ref_dispatch=True)
    use_kernel(kernel)
    net, l4, v = batch.eth_checksum_batch(to_dev(buf), batch.desc_to_device(desc, "cuda:0"), desc.size,
                                          flags=batch.F_REF_DISPATCH, mac=mac)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(net), wn)
    np.testing.assert_array_equal(u16(l4), wl)
