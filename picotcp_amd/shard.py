"""Frame-batch sharding across the GPUs of a node.

Frames are independent, so a batch splits into contiguous frame ranges, one per
rank; no collective touches the data path.  RCCL (torch.distributed "nccl")
carries only the start barrier and the max-over-ranks timing in bench.py.
"""
from __future__ import annotations


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """(first frame, frame count) of rank's contiguous shard; sizes differ by <= 1."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)
