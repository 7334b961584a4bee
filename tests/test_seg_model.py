"""CPU model of the segment pass's chunk locate (mchecksum_gpu_ext.hip:
seg_scan's per-segment object record, seg_locate's head test).

The scan writes, per segment s of object j, {j, first[j], first[j + 1], hs}
where hs is the object's head segment -- its first non-empty one -- when the
object starts in s's scan block and that block holds it, else "unknown".  The
chunk pass calls a chunk the object's head (it starts from the register init)
by `hs == s and off == 0` when hs is known and by `P[s] + off == P[first[j]]`
otherwise.  This checks, over random layouts with runs of empty segments,
empty objects, objects straddling small scan blocks and segments outside
every object, that the rule gives exactly one head chunk per non-empty object
and agrees with the byte-offset definition for every chunk.
"""
import random

import pytest

CHUNK = 256 << 10
NOOBJ = None


def scan_records(lens, first, blk):
    """seg_scan's record per segment, block by block (blk segments each)."""
    nseg, nobj = len(lens), len(first) - 1
    rec = [None] * nseg
    for s0 in range(0, nseg, blk):
        s1 = min(s0 + blk, nseg)
        for k in range(nobj):
            a0, a1 = first[k], first[k + 1]
            lo, hi = max(a0, s0), min(a1, s1)
            if lo >= hi:
                continue
            hs = NOOBJ
            if a0 >= s0:
                hs = next((i for i in range(lo, hi) if lens[i]), NOOBJ)
            for i in range(lo, hi):
                rec[i] = (k, a0, a1, hs)
    return rec


def heads(lens, first, blk):
    P = [0]
    for ln in lens:
        P.append(P[-1] + ln)
    rec = scan_records(lens, first, blk)
    found = {}
    for s, ln in enumerate(lens):
        if rec[s] is None:
            continue
        j, a0, _a1, hs = rec[s]
        for off in range(0, ln, CHUNK):
            by_offset = P[s] + off == P[a0]
            rule = (hs == s and off == 0) if hs is not NOOBJ else by_offset
            assert rule == by_offset, (s, off, rec[s])
            if rule:
                assert j not in found, j
                found[j] = s
    return found


@pytest.mark.parametrize("seed", range(40))
def test_head_rule_matches_byte_offsets(seed):
    rng = random.Random(seed)
    nseg = rng.randrange(1, 200)
    lens = [0 if rng.random() < 0.4 else rng.choice([1, 7, CHUNK - 1, CHUNK, CHUNK + 3, 3 * CHUNK]) for _ in range(nseg)]
    cuts = sorted(rng.randrange(0, nseg + 1) for _ in range(rng.randrange(1, 30)))
    first = [cuts[0]] + cuts[1:] + [max(cuts[-1], rng.randrange(cuts[-1], nseg + 1))]
    blk = rng.choice([1, 2, 3, 8, 1024])
    found = heads(lens, first, blk)
    for j in range(len(first) - 1):
        nonempty = any(lens[s] for s in range(first[j], first[j + 1]))
        assert (j in found) == nonempty, j


def test_heads_after_leading_empties_across_blocks():
    """The GPU test's layout (tests/test_gpu_ext.py) at block size 1024."""
    lens = [1] * 3200
    for s in list(range(1000, 1024)) + list(range(1030, 2053)) + [10, 11, 3070, 3071]:
        lens[s] = 0
    lens[2053] = 600000
    lens[12] = CHUNK + 7
    first = [0, 10, 20, 500, 1000, 1030, 2100, 2500, 3070, 3080, 3200]
    found = heads(lens, first, 1024)
    assert found[1] == 12 and found[4] == 1024 and found[5] == 2053 and found[8] == 3072
