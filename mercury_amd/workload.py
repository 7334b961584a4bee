"""Synthetic batch layouts of SURVEY.md 8(d), for bench.py and the tools.

Payload bytes are generated on the device (`gpu.fill_splitmix`); this module
only builds the host-side layout tables.  The variable-length (C4) layout:
len_i = 64 + splitmix64(seed ^ 0x4C454E4754480000 ^ i) % 65473, packed back to
back (offsets[0] = 0, offsets[i+1] = offsets[i] + len_i).  numpy, vectorised;
tests/test_workload.py pins it to the oracle's C generator.
"""
from __future__ import annotations

import numpy as np

LEN_SALT = 0x4C454E4754480000
_M64 = (1 << 64) - 1


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser over a uint64 array (wrapping arithmetic)."""
    z = np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def varlen_lengths(seed: int, count: int, min_len: int = 64, max_len: int = 65536) -> np.ndarray:
    if count < 0 or min_len > max_len:
        raise ValueError("bad length range")
    span = np.uint64(max_len - min_len + 1)
    idx = np.arange(count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        r = splitmix64(np.uint64((seed ^ LEN_SALT) & _M64) ^ idx)
    return np.uint64(min_len) + r % span


def varlen_offsets(seed: int, count: int, min_len: int = 64, max_len: int = 65536) -> np.ndarray:
    """count + 1 uint64 offsets of the packed variable-length batch."""
    off = np.zeros(count + 1, dtype=np.uint64)
    np.cumsum(varlen_lengths(seed, count, min_len, max_len), out=off[1:])
    return off


def segment_slots(seed: int, nseg: int) -> np.ndarray:
    """Bulk-segment layout (bench config "seg"): segment s of the batch lives in
    slot slots[s] of the buffer -- a seeded permutation, so an object's
    segments are scattered rather than adjacent."""
    return np.random.default_rng(seed & _M64).permutation(nseg)
