"""CPU tests of the N>1 path: contiguous frame sharding and the max-over-ranks
timing reduction bench.py uses, exercised with 2 gloo ranks."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from picotcp_amd.shard import shard_range


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 262144, 4194304, 1000003):
        for world in (1, 2, 3, 4, 8):
            seen = 0
            for r in range(world):
                first, cnt = shard_range(n, r, world)
                assert first == seen
                seen += cnt
            assert seen == n
            sizes = [shard_range(n, r, world)[1] for r in range(world)]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    from oracle import oracle as O
    from picotcp_amd import synth
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, ln = 1001, 1500
    buf = synth.uniform_batch(n, ln, seed=123)           # every rank sees the same global batch
    first, cnt = shard_range(n, rank, world)
    part = O.batch_uniform(buf[first * ln:], ln, ln, cnt)  # each rank checksums only its shard
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)                # bench.py's max-over-ranks
    parts = [None] * world
    dist.all_gather_object(parts, (first, part.tolist()))
    if rank == 0:
        full = np.zeros(n, dtype=np.uint16)
        for f, p in parts:
            full[f:f + len(p)] = p
        q.put((float(t[0]), bool(np.array_equal(full, O.batch_uniform(buf, ln, ln, n)))))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards_reassemble():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.spawn(_worker, args=(2, port, q), nprocs=2, join=True)
    tmax, ok = q.get(timeout=60)
    assert tmax == 2.0
    assert ok
