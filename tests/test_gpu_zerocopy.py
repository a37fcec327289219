"""GPU: zero-copy ingress (the batch form of pico_stack_recv_zerocopy, stack/pico_stack.c:479-527)
-- a burst in registered host memory, its descriptors and result arrays too, handed to the layer-2
device batch through pico_csum_host_device_pointer: the kernel reads the frames over PCIe where they
lie and writes the results (and, TX, the crc fields) straight into host memory; no staging copy.
Against the oracle."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import _lib, batch, synth

pytestmark = pytest.mark.gpu


def aligned(nbytes: int) -> np.ndarray:
    """A page-aligned uint8 host array."""
    raw = np.zeros(nbytes + 8192, np.uint8)
    a = (-raw.ctypes.data) % 4096
    return raw[a:a + nbytes]


class Registered:
    def __init__(self, *arrays):
        self.lib = _lib.load()
        self.arrays = arrays
        for a in arrays:
            _lib.check("pico_csum_host_register", self.lib.pico_csum_host_register(a.ctypes.data, a.nbytes))

    def dev(self, a) -> ctypes.c_void_p:
        p = self.lib.pico_csum_host_device_pointer(a.ctypes.data)
        assert p, self.lib.pico_csum_last_error()
        return ctypes.c_void_p(p)

    def close(self):
        for a in self.arrays:
            self.lib.pico_csum_host_unregister(a.ctypes.data)


@pytest.mark.parametrize("tx", [False, True])
def test_ipv4_zero_copy(tx):
    n = 20000
    lens = synth.imix_lengths(n, 12)
    b, net, avail = synth.ipv4_batch(lens, seed=13, proto=6, eth=True)
    buf = aligned(b.size)
    buf[:] = b
    d = batch.make_desc(net, avail)
    desc = aligned(d.nbytes)
    desc[:] = d.view(np.uint8)
    on, ol, v = aligned(2 * n), aligned(2 * n), aligned(n)
    before = buf.copy()
    reg = Registered(buf, desc, on, ol, v)
    try:
        lib = reg.lib
        fl = (batch.F_TX | batch.F_WRITE) if tx else 0
        rc = lib.pico_ipv4_checksum_batch_dev(reg.dev(buf), buf.size, reg.dev(desc), n, fl, reg.dev(on), reg.dev(ol),
                                              reg.dev(v), None)
        _lib.check("pico_ipv4_checksum_batch_dev", rc)
        torch.cuda.synchronize()
        wn, wl, wv = O.batch_ipv4(before, d, tx=tx)
        np.testing.assert_array_equal(v, wv)
        np.testing.assert_array_equal(on.view(np.uint16), wn)
        np.testing.assert_array_equal(ol.view(np.uint16), wl)
        if tx:                                           # the crc fields landed in host memory
            rn, rl, rv = O.batch_ipv4(buf, d)
            assert (rv == 1).all() and (rn == 0).all() and (rl == 0).all()
    finally:
        reg.close()

