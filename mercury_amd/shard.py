"""Partitioning a batch of independent payloads across ranks (one process per
GPU).  Payloads shard with no data exchange: a rank checksums
its own contiguous index range; the only collective is gathering the CRC
arrays afterwards (RCCL all_gather over xGMI on MI355X, gloo in CPU tests).
"""
from __future__ import annotations

import numpy as np


def fixed_shard(rank: int, world: int, total_count: int):
    """Contiguous payload range [first, first+count) of rank in a fixed-size batch
    of total_count payloads (the first total_count % world ranks get one more)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    q, r = divmod(total_count, world)
    first = rank * q + min(rank, r)
    return first, q + (1 if rank < r else 0)


def byte_balanced_cuts(offsets: np.ndarray, world: int) -> np.ndarray:
    """Cut an offsets table (count+1 entries) into world contiguous payload
    ranges of near-equal bytes: returns world+1 payload indices.  Rank r owns
    payloads [cuts[r], cuts[r+1]) -- the same rule the kernels use to split a
    variable-length batch between waves."""
    off = np.asarray(offsets, dtype=np.uint64)
    count = len(off) - 1
    total = int(off[-1] - off[0])
    cuts = np.empty(world + 1, dtype=np.int64)
    cuts[0], cuts[world] = 0, count
    for r in range(1, world):
        key = int(off[0]) + (total * r) // world
        cuts[r] = int(np.searchsorted(off[:count], np.uint64(key), side="left"))
    return cuts
