"""C4 on the HIP path: 4M x 1500 B frames, split into contiguous
`shard_range` shards exactly as bench.py's ranks split them, every shard through
pico_checksum_batch_uniform_dev, reassembled and compared with the oracle bit for bit.
Also the N>1 path with real ranks: 2 gloo processes sharing the one GPU, each
checksumming its shard with the HIP kernel."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from picotcp_amd import batch
from picotcp_amd.shard import shard_range

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _oracle_uniform(host: np.ndarray, ln: int, n: int) -> np.ndarray:
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    _, want = O.uniform_mt(host, ln, ln, n, threads, kind="port")
    return want


@pytest.mark.parametrize("world", [8, 3])
def test_c4_sharded_full_size(world):
    n, ln = 4194304, 1500                                   # 5.86 GiB of frames
    g = torch.Generator(device=DEV)
    g.manual_seed(4004 + world)
    frames = torch.randint(0, 256, (n * ln,), dtype=torch.uint8, device=DEV, generator=g)
    got = torch.empty(n, dtype=torch.int16, device=DEV)
    for r in range(world):
        first, cnt = shard_range(n, r, world)
        shard = frames[first * ln:(first + cnt) * ln]          # a rank's HBM holds only its shard
        batch.checksum_uniform(shard, ln, ln, cnt, out=got[first:first + cnt])
    torch.cuda.synchronize()
    got_h = got.cpu().numpy().view(np.uint16)
    host = frames.cpu().numpy()
    del frames
    torch.cuda.empty_cache()
    np.testing.assert_array_equal(got_h, _oracle_uniform(host, ln, n))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, ln = 65537, 1500
    g = torch.Generator()
    g.manual_seed(77)
    host = torch.randint(0, 256, (n * ln,), dtype=torch.uint8, generator=g)   # same global batch on every rank
    first, cnt = shard_range(n, rank, world)
    d = host[first * ln:(first + cnt) * ln].to(DEV)
    part = batch.checksum_uniform(d, ln, ln, cnt)          # the HIP kernel, not the oracle
    torch.cuda.synchronize()
    parts = [None] * world
    dist.all_gather_object(parts, (first, part.cpu().numpy().view(np.uint16).tolist()))
    if rank == 0:
        full = np.zeros(n, dtype=np.uint16)
        for f, p in parts:
            full[f:f + len(p)] = p
        want = O.batch_uniform(host.numpy(), ln, ln, n)
        q.put(bool(np.array_equal(full, want)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_hip_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_worker, args=(2, _free_port(), q), nprocs=2, join=True)
    assert q.get(timeout=60)
