"""Randomized differential tests: every batched kernel vs the oracle on random
descriptors, seeds, crc fields and fully random IPv4 / IPv6 header bytes (uint16
length wraps, IHL 0-15, options, truncated buffers, unknown protocols, fragments,
extension-header chains).  Seeded, so a failure reproduces.  Run on an MI355X with
`-m gpu`."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0)


def u16(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


# descriptor batches: the sorted-rounds kernel, automatic or with forced frames per wave
DESC_FPW = [None, 64, 33, 6, 5, 1]


def use_fpw(f):
    if f is None:
        batch.set_launch_override(0)
    else:
        batch.set_launch_override(2, fpw=f)


@pytest.mark.parametrize("trial", range(6))
def test_fuzz_raw_descriptors(trial):
    rng = np.random.default_rng(1000 + trial)
    size = int(rng.integers(1 << 16, 1 << 22))
    buf = synth.random_bytes(2000 + trial, size)
    n = int(rng.integers(1, 5000))
    kind = rng.random(n)
    lens = np.where(kind < 0.2, rng.integers(0, 8, n),
                    np.where(kind < 0.9, rng.integers(0, 2000, n), rng.integers(0, 70000, n))).astype(np.int64)
    lens = np.minimum(lens, size)
    offs = (rng.random(n) * (size - lens + 1)).astype(np.uint64)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) * (rng.random(n) < 0.5)
    desc = batch.make_desc(offs, lens, seeds)
    crc = int(rng.choice([-1, 0, 2, 10, 16, 6]))
    want = O.batch_raw(buf, desc, crc_off=crc)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc, DEV)
    for shape in DESC_FPW:
        use_fpw(shape)
        got = u16(batch.checksum_batch(d_buf, d_desc, n, crc_off=crc))
        np.testing.assert_array_equal(got, want, err_msg=f"trial={trial} shape={shape} crc={crc}")


def random_datagrams(rng, n, ipv6: bool):
    """Packed datagrams whose header bytes are random except where a coin flip makes
    them plausible (so both the malformed and the valid paths are exercised)."""
    lens = rng.integers(0, 1600, n).astype(np.int64)
    small = rng.random(n) < 0.05
    lens[small] = rng.integers(0, 60, int(small.sum()))
    starts = np.zeros(n, dtype=np.int64)
    starts[1:] = np.cumsum(lens + rng.integers(0, 3, n))[:-1]
    size = int(starts[-1] + lens[-1] + 64)
    buf = synth.random_bytes(int(rng.integers(0, 1 << 30)), size)
    seeds = np.zeros(n, dtype=np.uint32)
    for i in range(n):
        o, L = int(starts[i]), int(lens[i])
        if rng.random() < 0.7 and L >= 40:          # plausible header
            if not ipv6:
                ihl = int(rng.choice([5, 5, 5, 6, 15, 3]))
                buf[o] = 0x40 | ihl
                tot = L if rng.random() < 0.8 else int(rng.integers(0, 65536))
                buf[o + 2], buf[o + 3] = tot >> 8, tot & 0xFF
                buf[o + 9] = int(rng.choice([6, 17, 1, 6, 47]))
            else:
                buf[o] = 0x60
                pl = L - 40 if rng.random() < 0.8 else int(rng.integers(0, 65536))
                buf[o + 4], buf[o + 5] = (pl >> 8) & 0xFF, pl & 0xFF
                buf[o + 6] = int(rng.choice([6, 17, 58, 6, 0, 43]))
                if rng.random() < 0.2:
                    seeds[i] = int(rng.choice([48, 40, 56, 30, 2000])) | (int(rng.choice([6, 17, 58])) << 16)
    avail = np.maximum(lens + rng.integers(-8, 9, n), 0)
    avail = np.minimum(avail, size - starts).astype(np.uint32)
    d = batch.make_desc(starts.astype(np.uint64), avail, seeds)
    return buf, d


@pytest.mark.parametrize("trial", range(4))
@pytest.mark.parametrize("tx", [False, True])
def test_fuzz_ipv4(trial, tx):
    rng = np.random.default_rng(3000 + trial)
    n = int(rng.integers(200, 3000))
    buf, desc = random_datagrams(rng, n, ipv6=False)
    desc["seed"] = 0
    wn, wl, wv = O.batch_ipv4(buf, desc, tx=tx)
    d_desc = batch.desc_to_device(desc, DEV)
    for shape in (None, 64, 3, 1):
        use_fpw(shape)
        net, l4, v = batch.ipv4_checksum_batch(to_dev(buf), d_desc, n, flags=batch.F_TX if tx else 0)
        np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"verdict trial={trial} shape={shape}")
        np.testing.assert_array_equal(u16(net), wn, err_msg=f"net trial={trial} shape={shape}")
        np.testing.assert_array_equal(u16(l4), wl, err_msg=f"l4 trial={trial} shape={shape}")


@pytest.mark.parametrize("trial", range(4))
@pytest.mark.parametrize("tx", [False, True])
def test_fuzz_ipv6(trial, tx):
    rng = np.random.default_rng(4000 + trial)
    n = int(rng.integers(200, 3000))
    buf, desc = random_datagrams(rng, n, ipv6=True)
    wl, wv = O.batch_ipv6(buf, desc, tx=tx)
    d_desc = batch.desc_to_device(desc, DEV)
    for shape in (None, 64, 7, 1):
        use_fpw(shape)
        l4, v = batch.ipv6_checksum_batch(to_dev(buf), d_desc, n, flags=batch.F_TX if tx else 0)
        np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"verdict trial={trial} shape={shape}")
        np.testing.assert_array_equal(u16(l4), wl, err_msg=f"l4 trial={trial} shape={shape}")
    if not tx:                                   # the next-header dispatch on the same bytes
        wl, wv = O.batch_ipv6(buf, desc, nxthdr_dispatch=True)
        l4, v = batch.ipv6_checksum_batch(to_dev(buf), d_desc, n, flags=batch.F_NXTHDR_DISPATCH)
        np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"nx verdict trial={trial}")
        np.testing.assert_array_equal(u16(l4), wl, err_msg=f"nx l4 trial={trial}")


@pytest.mark.parametrize("trial", range(3))
def test_fuzz_rx_chains(trial):
    """make_ref_rx.py's generators (the reference-pinned families: fragments, the evil bit,
    IHL < 5, bad sources; random IPv6 extension-header chains for the kernel's own walk),
    fresh seeds, against the oracle -- which those fixtures pin to the compiled reference."""
    from tests.golden import make_ref_rx as M
    rng = np.random.default_rng(9100 + trial)
    for gen, fam in ((M.gen_v4, 4), (M.gen_v6, 6)):
        items = gen(rng, 3000)
        buf, off, av = M.pack(items, rng)
        desc = batch.make_desc(off, av)
        d_desc = batch.desc_to_device(desc, DEV)
        for shape in (None, 64, 5):
            use_fpw(shape)
            if fam == 4:
                wn, wl, wv = O.batch_ipv4(buf, desc)
                net, l4, v = batch.ipv4_checksum_batch(to_dev(buf), d_desc, len(items))
                np.testing.assert_array_equal(u16(net), wn, err_msg=f"v4 net trial={trial} shape={shape}")
            else:
                wl, wv = O.batch_ipv6(buf, desc)
                l4, v = batch.ipv6_checksum_batch(to_dev(buf), d_desc, len(items))
            np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"v{fam} verdict trial={trial} shape={shape}")
            np.testing.assert_array_equal(u16(l4), wl, err_msg=f"v{fam} l4 trial={trial} shape={shape}")


@pytest.mark.parametrize("trial", range(4))
def test_fuzz_uniform(trial):
    rng = np.random.default_rng(5000 + trial)
    ln = int(rng.choice([0, 1, 3, 20, 64, 353, 1500, 1501, 4096, 9000, 20001]))
    stride = ln + int(rng.integers(0, 40))
    n = int(rng.integers(1, 20000 if ln < 5000 else 800))
    buf = synth.uniform_batch(n, ln, max(stride, 1), seed=6000 + trial)
    if buf.size == 0:
        buf = np.zeros(16, np.uint8)
    seed = int(rng.integers(0, 1 << 32))
    want = O.batch_uniform(buf, max(stride, 1), ln, n, seed)
    d = to_dev(buf)
    for shape in (None, (4, 8, 16, 1, 1, 2), (16, 8, 8, 1, 2, 2), (64, 4, 4, 2, 2, 1), (8, 2, 8, 4, 1, 1)):
        if shape is None:
            batch.set_launch_override(0)
        else:
            batch.set_launch_override(shape[0], shape[1], shape[2], shape[3], shape[4], shape[5])
        got = u16(batch.checksum_uniform(d, max(stride, 1), ln, n, seed=seed))
        np.testing.assert_array_equal(got, want, err_msg=f"trial={trial} ln={ln} shape={shape}")
