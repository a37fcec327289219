"""GPU: TX through the batches, checked against the frames the compiled reference stack emits
(tests/golden/ref_tx_cases.npz, tests/test_ref_tx.py): their crc fields scrambled, run through
pico_ipv4_checksum_batch_dev and pico_eth_checksum_batch_dev with F_TX | F_WRITE -- packed back to
back at every alignment, one per 2 KiB slot, and behind Ethernet headers -- every byte written must
be the reference's, and nothing else may change."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from picotcp_amd import batch
from tests.test_gpu_parity import to_dev
from tests.test_ref_tx import fixture, scrambled

pytestmark = pytest.mark.gpu

MAC = bytes.fromhex("02005e0a0b0c")


def layout(buf, off, lens, shift, slot, l2):
    """The datagrams re-laid: `shift` bytes in, back to back (slot 0) or one per slot, each behind
    l2 bytes of Ethernet header (l2 0 or 14).  Returns (bytes, datagram offsets)."""
    n = lens.size
    step = [slot] * n if slot else [l2 + int(x) for x in lens]
    starts = shift + np.concatenate([[0], np.cumsum(step[:-1])]).astype(np.int64)
    out = np.zeros(int(starts[-1]) + l2 + int(lens[-1]) + 64, np.uint8)
    for i in range(n):
        o = int(off[i])
        out[starts[i] + l2:starts[i] + l2 + lens[i]] = buf[o:o + lens[i]]
        if l2:
            out[starts[i]:starts[i] + 14] = np.frombuffer(MAC + bytes(6) + b"\x08\x00", np.uint8)
    return out, (starts + l2).astype(np.uint64)


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 7])
@pytest.mark.parametrize("slot", [0, 2048])
@pytest.mark.parametrize("l2", [0, 14])
@pytest.mark.parametrize("reps", [1, 64])
def test_tx_writes_reference_bytes(shift, slot, l2, reps):
    buf, off, lens, proto = fixture()
    if reps > 1:                                             # a burst large enough for the stream waves
        n0 = lens.size
        buf = np.tile(buf, reps)
        off = (off[None, :] + (np.arange(reps, dtype=np.uint64) * np.uint64(buf.size // reps))[:, None]).reshape(-1)
        lens, proto = np.tile(lens, reps), np.tile(proto, reps)
        assert lens.size == n0 * reps
    want, noff = layout(buf, off, lens, shift, slot, l2)
    src, _ = layout(scrambled(buf, off, proto, 11 + shift), off, lens, shift, slot, l2)
    d = to_dev(src)
    if l2:
        desc = batch.desc_to_device(batch.make_desc(noff - np.uint64(14), lens + 14), "cuda:0")
        _, _, v = batch.eth_checksum_batch(d, desc, lens.size, flags=batch.F_TX | batch.F_WRITE)
    else:
        desc = batch.desc_to_device(batch.make_desc(noff, lens), "cuda:0")
        _, _, v = batch.ipv4_checksum_batch(d, desc, lens.size, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    assert (v.cpu().numpy() & 0x7F == 1).all()
    got = d.cpu().numpy()
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} bytes differ from the reference's frames, first at {bad[:8]}"
