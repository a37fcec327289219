"""GPU: the reassembly flat grid's library scratch (pico_csum_k_frag.hip reasm_scratch) is
returned when the calling thread exits and on pico_csum_release_thread_scratch -- a driver that
runs bursts on short-lived worker threads does not accumulate device memory."""
from __future__ import annotations

import threading

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import _lib, batch
from tests import golden_data as G
from tests.test_gpu_frag import layout
from tests.test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu

# 256K one-fragment datagrams (IPv4/UDP, 8 transport bytes, UDP crc 0): each thread's flat-grid
# scratch is 256K x 8 B x 1.5 = 3 MiB, so 32 leaked buffers would be 96 MiB
N = 256 * 1024
_CASE = []


def _case():
    if not _CASE:
        _CASE.append(_make())
    return _CASE[0]


def _make():
    per = 14 + 20 + 8
    buf = np.zeros(N * per + 16, np.uint8)
    net = np.arange(N, dtype=np.int64) * per + 14
    h = np.zeros((N, 28), np.uint8)
    h[:, 0], h[:, 3], h[:, 8], h[:, 9] = 0x45, 28, 64, 17
    h[:, 4], h[:, 5] = (np.arange(N) >> 8) & 0xFF, np.arange(N) & 0xFF
    h[:, 12:16] = [10, 0, 0, 1]
    h[:, 16:20] = [10, 0, 0, 2]
    h[:, 24], h[:, 25] = 0, 8                            # UDP length 8, crc 0 (not verified)
    buf[(net[:, None] + np.arange(28)[None, :]).reshape(-1)] = h.reshape(-1)
    d = G.ipv4_desc(net.astype(np.uint64), np.full(N, 28, np.uint32))
    grp = np.stack([np.arange(N), np.ones(N)], 1).astype(np.uint32)
    od, size = layout([8] * N, shift=4)
    want = O.ipv4_reassemble(buf, d, grp, np.zeros(size, np.uint8), od)
    assert (want[2] == 1).all()
    dev = (to_dev(buf), to_dev(d.view(np.uint8)), d.size,
           to_dev(np.ascontiguousarray(grp, np.uint32).reshape(-1).view(np.int32)), to_dev(od.view(np.uint8)))
    return dev, size, want


def _run(dev, out, res, stream):
    b, d, nf, grp, od_d = dev
    with torch.cuda.stream(stream):
        batch.ipv4_reassemble_batch(b, d, nf, grp, out, od_d, stream=stream, results=res)
    stream.synchronize()


def _free():
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info()[0]


def test_thread_exit_frees_scratch():
    dev, size, want = _case()
    k = 32
    outs = [torch.zeros(size, dtype=torch.uint8, device="cuda:0") for _ in range(k)]
    res = [(torch.zeros(N, dtype=torch.int32, device="cuda:0"), torch.zeros(N, dtype=torch.int16, device="cuda:0"),
            torch.zeros(N, dtype=torch.uint8, device="cuda:0")) for _ in range(k)]
    streams = [torch.cuda.Stream() for _ in range(k)]
    _run(dev, outs[0], res[0], streams[0])               # the main thread's own scratch, before the baseline
    errs = []

    def worker(i):
        try:
            _run(dev, outs[i], res[i], streams[i])
        except Exception as e:                            # noqa: BLE001 (reported below)
            errs.append(e)

    def threads():
        for i in range(k):                                # short-lived threads, one after another
            t = threading.Thread(target=worker, args=(i,))
            t.start()
            t.join()

    # the HIP runtime keeps some memory per thread it has served (~1.25 MiB, reused by later
    # threads): a first round of threads settles it, the second is measured
    threads()
    free0 = _free()
    threads()
    assert not errs, errs
    free1 = _free()
    assert free0 - free1 < (1 << 20), f"{(free0 - free1) / 2**20:.1f} MiB not returned after {k} threads exited"
    for r in res:                                         # and every thread's results were right
        np.testing.assert_array_equal(r[2].cpu().numpy(), want[2])
        np.testing.assert_array_equal(r[0].cpu().numpy().view(np.uint32), want[0])


def test_release_thread_scratch():
    dev, size, want = _case()
    out = torch.zeros(size, dtype=torch.uint8, device="cuda:0")
    res = (torch.zeros(N, dtype=torch.int32, device="cuda:0"), torch.zeros(N, dtype=torch.int16, device="cuda:0"),
           torch.zeros(N, dtype=torch.uint8, device="cuda:0"))
    s = torch.cuda.Stream()
    lib = _lib.load()
    assert lib.pico_csum_release_thread_scratch() == 0
    free0 = _free()
    _run(dev, out, res, s)
    free1 = _free()
    assert lib.pico_csum_release_thread_scratch() == 0
    free2 = _free()
    assert free0 - free1 >= N * 8, "the flat grid allocated no scratch"
    assert abs(free0 - free2) < (1 << 20), "pico_csum_release_thread_scratch did not return the scratch"
    np.testing.assert_array_equal(res[2].cpu().numpy(), want[2])
    _run(dev, out, res, s)                                # allocates again
    np.testing.assert_array_equal(res[2].cpu().numpy(), want[2])
