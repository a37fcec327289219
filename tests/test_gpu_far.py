"""Fused IPv4 / IPv6 batches whose datagrams lie far apart in a batch over 2 GiB: one
wave's 64 frames span > 1 GiB, so the phase-1 head-window buffer loads (sorted_batch in
picotcp_amd/csrc/pico_csum_kernels.hip, a window of at most 2 GiB from 1 GiB below the
wave's first frame) cover only some of them and the rest take the branched second pass.
Checked bit for bit against the oracle on the same datagrams packed densely.
Run on an MI355X with `-m gpu`."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch
from tests.test_gpu_fuzz import random_datagrams, u16

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0)


@pytest.mark.parametrize("ipv6", [False, True])
def test_far_apart_over_2gib(ipv6):
    rng = np.random.default_rng(7000 + ipv6)
    n = 96
    buf, desc = random_datagrams(rng, n, ipv6=ipv6)
    if not ipv6:
        desc["seed"] = 0
    big_n = 9 << 28                                      # 2.25 GiB
    spacing = (big_n - 4096) // n                        # ~24 MB: a 64-frame wave spans ~1.5 GiB
    far = desc.copy()
    far["off"] = np.arange(n, dtype=np.uint64) * np.uint64(spacing) + rng.integers(0, 16, n).astype(np.uint64)
    big = torch.zeros(big_n, dtype=torch.uint8, device=DEV)
    for i in range(n):
        o, ln, t = int(desc["off"][i]), int(desc["len"][i]), int(far["off"][i])
        if ln:
            big[t:t + ln] = torch.from_numpy(buf[o:o + ln].copy()).to(DEV)
    d_desc = batch.desc_to_device(far, DEV)
    for tx in (False, True):
        fl = batch.F_TX if tx else 0
        for shape in (None, 64, 7):
            if shape is None:
                batch.set_launch_override(0)
            else:
                batch.set_launch_override(2, fpw=shape)
            msg = f"ipv6={ipv6} tx={tx} shape={shape}"
            if ipv6:
                wl, wv = O.batch_ipv6(buf, desc, tx=tx)
                l4, v = batch.ipv6_checksum_batch(big, d_desc, n, flags=fl)
            else:
                wn, wl, wv = O.batch_ipv4(buf, desc, tx=tx)
                net, l4, v = batch.ipv4_checksum_batch(big, d_desc, n, flags=fl)
                np.testing.assert_array_equal(u16(net), wn, err_msg="net " + msg)
            np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg="verdict " + msg)
            np.testing.assert_array_equal(u16(l4), wl, err_msg="l4 " + msg)
    del big
    torch.cuda.empty_cache()


def test_nat_far_apart_over_2gib():
    """The NAT batch on the same far layout: frames outside the wave's window read their old port
    from memory (not the LDS stage) and are translated like any other."""
    rng = np.random.default_rng(7100)
    n = 96
    buf, desc = random_datagrams(rng, n, ipv6=False)
    desc["seed"] = 0
    for o, ln in zip(desc["off"].astype(np.int64), desc["len"]):
        if ln >= 8:
            buf[o + 6], buf[o + 7] = 0x40, 0                # DF, no fragment: NAT's datagrams
    nat = np.zeros(n, O.NAT_DTYPE)
    nat["addr"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    nat["port"] = rng.integers(0, 1 << 16, n).astype(np.uint16)
    nat["dir"] = rng.choice(np.array([1, 2], np.uint8), n)
    big_n = 9 << 28                                      # 2.25 GiB
    spacing = (big_n - 4096) // n
    far = desc.copy()
    far["off"] = np.arange(n, dtype=np.uint64) * np.uint64(spacing) + rng.integers(0, 16, n).astype(np.uint64)
    want_buf = buf.copy()
    wn, wl, wv = O.batch_ipv4_nat(want_buf, desc, nat)
    assert (wv == 1).sum() > 15
    d_nat = torch.from_numpy(nat.view(np.uint8)).to(DEV)
    d_desc = batch.desc_to_device(far, DEV)
    big = torch.zeros(big_n, dtype=torch.uint8, device=DEV)
    for shape in (None, 64, 7):
        for i in range(n):
            o, ln, t = int(desc["off"][i]), int(desc["len"][i]), int(far["off"][i])
            if ln:
                big[t:t + ln] = torch.from_numpy(buf[o:o + ln].copy()).to(DEV)
        if shape is None:
            batch.set_launch_override(0)
        else:
            batch.set_launch_override(2, fpw=shape)
        net, l4, v = batch.ipv4_nat_batch(big, d_desc, n, d_nat)
        torch.cuda.synchronize()
        msg = f"shape={shape}"
        np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg="verdict " + msg)
        np.testing.assert_array_equal(u16(net), wn, err_msg="net " + msg)
        np.testing.assert_array_equal(u16(l4), wl, err_msg="l4 " + msg)
        for i in range(n):
            o, ln, t = int(desc["off"][i]), int(desc["len"][i]), int(far["off"][i])
            if ln:
                np.testing.assert_array_equal(big[t:t + ln].cpu().numpy(), want_buf[o:o + ln], err_msg=f"bytes {i} {msg}")
    del big
    torch.cuda.empty_cache()
