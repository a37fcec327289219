"""GPU: host-resident descriptor batches on a burst the device addresses directly (page-locked by
hipHostMalloc, or registered with pico_csum_host_register): the kernel reads -- and with F_WRITE
writes -- the burst in place through its device alias, only descriptors and results staged
(pico_csum.c desc_batch_in_place).  Against the oracle and against the staged path on the same
burst (pico_csum_set_host_in_place(0)), with a staging size that makes every burst several
chunks."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import _lib, batch, synth
from tests import golden_data as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hb():
    h = batch.HostBatch(0, staging_bytes=1 << 20)         # 1 MiB: 16K descriptors a chunk in place
    yield h
    h.close()


@pytest.fixture(autouse=True)
def _reset():
    yield
    batch.set_host_in_place(True)


def pinned(a: np.ndarray):
    """A page-locked copy of `a` (the tensor keeps the memory alive)."""
    t = torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
    return t, t.numpy()


def both_paths(call):
    """The call in place, then staged (the knob off), on fresh copies made by `call`."""
    batch.set_host_in_place(True)
    a = call()
    batch.set_host_in_place(False)
    b = call()
    batch.set_host_in_place(True)
    return a, b


def test_ipv4_rx_tx_in_place(hb):
    lens = synth.imix_lengths(60_000, 41)
    buf, net, avail = synth.ipv4_batch(lens, seed=41, proto=6)
    d = batch.make_desc(net, avail)
    keep, pb = pinned(buf)
    for tx in (False, True):
        on, ol, v = hb.ipv4_checksum_batch(pb, d, flags=_lib.F_TX if tx else 0)
        wn, wl, wv = O.batch_ipv4(buf, d, tx=tx)
        np.testing.assert_array_equal(v, wv)
        np.testing.assert_array_equal(on, wn)
        np.testing.assert_array_equal(ol, wl)
    # TX written in place: the same bytes as the staged path writes back
    def write():
        k, p = pinned(buf)
        hb.ipv4_checksum_batch(p, d, flags=_lib.F_TX | _lib.F_WRITE)
        return p.copy()
    a, b = both_paths(write)
    np.testing.assert_array_equal(a, b)
    assert np.count_nonzero(a != buf) > d.size          # (the crc fields were written)
    k2, p2 = pinned(a)
    on, ol, v = hb.ipv4_checksum_batch(p2, d)
    assert (v == 1).all() and (on == 0).all() and (ol == 0).all()


def test_unsorted_and_out_of_bounds_in_place(hb):
    lens = synth.imix_lengths(20_000, 43)
    buf, net, avail = synth.ipv4_batch(lens, seed=43, proto=6)
    d = batch.make_desc(net, avail)
    d = d[np.random.default_rng(4).permutation(d.size)]
    d["off"][::97] = buf.size + 5
    d["len"][1::101] = buf.size
    keep, pb = pinned(buf)
    a, b = both_paths(lambda: hb.ipv4_checksum_batch(pb, d))
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    oob = (d["off"] > buf.size) | (d["len"].astype(np.uint64) > buf.size - np.minimum(d["off"], buf.size))
    assert oob.sum() > 300 and (a[2][oob] == 8).all()
    wn, wl, wv = O.batch_ipv4(buf, d[~oob])
    np.testing.assert_array_equal(a[2][~oob], wv)
    np.testing.assert_array_equal(a[0][~oob], wn)


def test_ipv6_eth_raw_in_place(hb):
    c6 = G.ipv6_cases()
    k6, b6 = pinned(c6["buf"])
    ol, v = hb.ipv6_checksum_batch(b6, G.ipv6_desc(c6))
    np.testing.assert_array_equal(ol, c6["rx_l4"])
    np.testing.assert_array_equal(v, c6["rx_verdict"])
    ce = G.eth_cases()
    ke, be = pinned(ce["buf"])
    on, ol, v = hb.eth_checksum_batch(be, G.eth_desc(ce), mac=ce["mac"].tobytes())
    np.testing.assert_array_equal(on, ce["rx_net"])
    np.testing.assert_array_equal(ol, ce["rx_l4"])
    np.testing.assert_array_equal(v, ce["rx_verdict"])
    # raw with the crc stored in place
    n = 30_000
    rng = np.random.default_rng(19)
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 3)[:-1]]).astype(np.uint64)
    raw = synth.random_bytes(78, int(offs[-1]) + int(lens[-1]) + 8)
    d = batch.make_desc(offs, lens, rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32))
    want = O.batch_raw(raw, d, crc_off=2)
    kr, br = pinned(raw)
    out = hb.checksum_batch(br, d, crc_off=2, flags=_lib.F_WRITE)
    np.testing.assert_array_equal(out, want)
    has = lens >= 4
    o = offs[has].astype(np.int64)
    np.testing.assert_array_equal((br[o + 2].astype(np.uint16) << 8) | br[o + 3], want[has])


def test_registered_numpy_burst(hb):
    """A plain numpy burst registered with pico_csum_host_register is read in place; unregistered,
    the same call takes the staged path -- same results."""
    lens = synth.imix_lengths(30_000, 47)
    buf, net, avail = synth.ipv4_batch(lens, seed=47, proto=6)
    d = batch.make_desc(net, avail)
    lib = _lib.load()
    ptr = ctypes.c_void_p(buf.ctypes.data)
    _lib.check("pico_csum_host_register", lib.pico_csum_host_register(ptr, buf.nbytes))
    try:
        assert lib.pico_csum_host_device_pointer(ptr)
        a = hb.ipv4_checksum_batch(buf, d)
    finally:
        _lib.check("pico_csum_host_unregister", lib.pico_csum_host_unregister(ptr))
    b = hb.ipv4_checksum_batch(buf, d)
    wn, wl, wv = O.batch_ipv4(buf, d)
    for x, y, w in zip(a, b, (wn, wl, wv)):
        np.testing.assert_array_equal(x, w)
        np.testing.assert_array_equal(y, w)


def test_all_pinned_is_one_zero_copy_launch(hb):
    """Burst, descriptors and result arrays all page-locked (a driver's pinned rings): one launch on
    their device aliases, nothing staged -- TX written in place too."""
    lens = synth.imix_lengths(50_000, 53)
    buf, net, avail = synth.ipv4_batch(lens, seed=53, proto=6)
    d = batch.make_desc(net, avail)
    kb, pb = pinned(buf)
    kd = torch.from_numpy(np.ascontiguousarray(d).view(np.uint8).copy()).pin_memory()
    pd = kd.numpy().view(batch.DESC_DTYPE)
    assert pd.ctypes.data % 16 == 0
    outs = [torch.zeros(d.size, dtype=dt).pin_memory() for dt in (torch.int16, torch.int16, torch.uint8)]
    po = (outs[0].numpy().view(np.uint16), outs[1].numpy().view(np.uint16), outs[2].numpy())
    for tx in (False, True):
        on, ol, v = hb.ipv4_checksum_batch(pb, pd, flags=_lib.F_TX if tx else 0, out=po)
        assert on is po[0]
        wn, wl, wv = O.batch_ipv4(buf, d, tx=tx)
        np.testing.assert_array_equal(v, wv)
        np.testing.assert_array_equal(on, wn)
        np.testing.assert_array_equal(ol, wl)
    hb.ipv4_checksum_batch(pb, pd, flags=_lib.F_TX | _lib.F_WRITE, out=po)
    kr, ref = pinned(buf)
    batch.set_host_in_place(False)
    hb.ipv4_checksum_batch(ref, d, flags=_lib.F_TX | _lib.F_WRITE)
    batch.set_host_in_place(True)
    np.testing.assert_array_equal(pb, ref)
    on, ol, v = hb.ipv4_checksum_batch(pb, pd, out=po)
    assert (v == 1).all() and (on == 0).all() and (ol == 0).all()


def test_frame_larger_than_staging_in_place(hb):
    """No frame is staged on the in-place path: a 2 MiB frame with 1 MiB of staging is summed (the
    staged path refuses it, tests/test_gpu_host_desc.py)."""
    raw = synth.random_bytes(91, 3 << 20)
    d = batch.make_desc([5, 1 << 20], [2 << 20, 777], [0, 0])
    kr, br = pinned(raw)
    out = hb.checksum_batch(br, d)
    np.testing.assert_array_equal(out, O.batch_raw(raw, d))
    batch.set_host_in_place(False)
    with pytest.raises(_lib.PicoCsumError) as e:
        hb.checksum_batch(br, d)
    assert e.value.rc == -_lib.EINVAL


def test_knob_rejects_bad_mode():
    with pytest.raises(_lib.PicoCsumError):
        _lib.check("pico_csum_set_host_in_place", _lib.load().pico_csum_set_host_in_place(2))
