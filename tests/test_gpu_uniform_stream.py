"""GPU: uniform rings on the stream waves (csum_uniform_stream_kernel in pico_csum_k_sorted.hip) --
frame i at base + i * stride; wave w reads frames [w R, w R + R) as one span in address order and
lane j takes the prefixes at both ends of frames j, j + 64, ... as they pass.

Forced on (pico_csum_set_uniform_stream) at several frames-per-wave R (1, below 64, 64 and
multiples, the automatic one), against the oracle bit for bit: C1's 1500-byte frames, C3's 9000,
odd lengths, gaps between frames, odd frame starts (the byte-swapped fold) with the largest seed
the host allows there, even starts with any seed (the uint32 accumulator wraps exactly as the
reference's), 64 KiB frames; plus the host's choice of kernel: small, sparse and odd-start rings
with a seed that could carry take the lane-group kernels, with the same results."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset_shape():
    yield
    batch.set_uniform_stream(0, 0)


def ring(n, stride, length, shift, seed):
    g = torch.Generator(device="cuda:0")
    g.manual_seed(seed)
    buf = torch.randint(0, 256, ((n - 1) * stride + length + shift + 64,), dtype=torch.uint8, device="cuda:0",
                        generator=g)
    return buf


def check(n, stride, length, shift=0, seed=0, mode=1, fpw=0, zero_some=False):
    buf = ring(n, stride, length, shift, n + stride + length + shift)
    if zero_some:                                          # all-zero frames: the fold keeps zero
        buf[shift:shift + 3 * stride] = 0
    batch.set_uniform_stream(mode, fpw)
    view = buf[shift:]
    got = batch.checksum_uniform(view, stride, length, n, seed=seed)
    torch.cuda.synchronize()
    want = O.batch_uniform(view.cpu().numpy(), stride, length, n, seed)
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint16), want)


@pytest.mark.parametrize("mode,fpw", [(0, 0), (1, 0), (1, 64), (1, 128), (1, 256), (1, 16), (1, 3), (1, 1), (1, 1000)])
def test_c1_frames(mode, fpw):
    check(262144, 1500, 1500, mode=mode, fpw=fpw)


@pytest.mark.parametrize("mode,fpw", [(0, 0), (1, 64), (1, 300), (1, 7)])
def test_c3_frames(mode, fpw):
    check(65536, 9000, 9000, mode=mode, fpw=fpw)


@pytest.mark.parametrize("length,stride", [(64, 64), (1, 1), (2, 2), (63, 63), (1500, 1536), (9000, 9000),
                                           (1499, 1500), (4097, 4100)])
@pytest.mark.parametrize("shift", [0, 1])
def test_lengths_gaps_and_odd_starts(length, stride, shift):
    n = 40000 if length < 4000 else 12000
    check(n, stride, length, shift=shift, seed=0x7FFFFFFF if (shift | stride) & 1 else 0xFFFFFFFF, fpw=100,
          zero_some=True)


@pytest.mark.parametrize("shift,seed", [(0, 0xFFFFFFFF), (0, 0x12345678), (1, 0x7FFFFFFF), (1, 0)])
def test_64k_frames(shift, seed):
    # 65535 at an odd start: the largest the fold allows; 65536 at even starts (the uint32 wrap)
    length = 65535 if shift else 65536
    check(2600, length, length, shift=shift, seed=seed, fpw=3)


@pytest.mark.parametrize("length,stride,shift,seed", [(1500, 4096, 0, 0), (1500, 1500, 1, 0x80000000),
                                                      (70000, 70000, 1, 5)])
def test_host_picks_lane_group_kernels(length, stride, shift, seed):
    """Sparse rings, odd starts with a seed that could carry: the other kernels, same results."""
    check(6000 if length < 10000 else 1500, stride, length, shift=shift, seed=seed, fpw=64)


@pytest.mark.parametrize("mode,fpw", [(1, 128), (1, 16)])
def test_repeat_and_graph(mode, fpw):
    n, ln = 262144, 1500
    buf = ring(n, ln, ln, 0, 3)
    want = O.batch_uniform(buf.cpu().numpy(), ln, ln, n, 0)
    batch.set_uniform_stream(mode, fpw)
    outs = [torch.empty(n, dtype=torch.int16, device="cuda:0") for _ in range(3)]
    for o in outs:
        batch.checksum_uniform(buf, ln, ln, n, out=o)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for o in outs:
                batch.checksum_uniform(buf, ln, ln, n, out=o)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        for o in outs:
            o.zero_()
        g.replay()
        torch.cuda.synchronize()
        for o in outs:
            np.testing.assert_array_equal(o.cpu().numpy().view(np.uint16), want)
