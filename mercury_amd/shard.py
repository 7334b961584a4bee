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


class ShardPlan:
    """One rank's share of a global batch, as bench.py lays it out in HBM.

    first, count  -- global payload range [first, first + count) of this rank
    counts        -- payloads per rank (all ranks; all_gather pads to the max)
    byte_base     -- global byte offset of this rank's buffer (a multiple of 8,
                     so the synthetic splitmix64 words line up: first_word =
                     byte_base // 8)
    nbytes        -- bytes of the rank's buffer (its payloads, plus the leading
                     partial word of a byte-packed batch)
    offsets       -- offsets table of the rank's payloads relative to byte_base
                     (count + 1 entries), or None for a fixed-size batch
    """

    def __init__(self, first, count, counts, byte_base, nbytes, offsets=None):
        self.first, self.count, self.counts = int(first), int(count), [int(c) for c in counts]
        self.byte_base, self.nbytes, self.offsets = int(byte_base), int(nbytes), offsets

    @property
    def first_word(self) -> int:
        return self.byte_base // 8

    @property
    def firsts(self):
        return [int(x) for x in np.concatenate([[0], np.cumsum(self.counts)[:-1]])]


def batch_shard(rank: int, world: int, global_count: int, length: int | None = None,
                offsets_global: np.ndarray | None = None) -> ShardPlan:
    """Rank's contiguous share of ONE global batch: equal payload counts for a
    fixed-size batch (fixed_shard), equal bytes for a byte-packed offsets batch
    (byte_balanced_cuts).  No data moves between ranks: each rank generates or
    holds exactly its own bytes."""
    if offsets_global is None:
        if length is None or length % 8:
            raise ValueError("fixed batches need a payload length that is a multiple of 8")
        spans = [fixed_shard(r, world, global_count) for r in range(world)]
        first, count = spans[rank]
        return ShardPlan(first, count, [c for _, c in spans], first * length, count * length)
    off = np.asarray(offsets_global, dtype=np.uint64)
    if len(off) != global_count + 1:
        raise ValueError("offsets_global must hold global_count + 1 entries")
    cuts = byte_balanced_cuts(off, world)
    first, last = int(cuts[rank]), int(cuts[rank + 1])
    base = int(off[first]) // 8 * 8
    local = (off[first:last + 1] - np.uint64(base)).astype(np.uint64)
    return ShardPlan(first, last - first, np.diff(cuts).tolist(), base, int(off[last]) - base, local)
