"""CPU model of the balanced static split's unit iterator (crc_gpu_device.h,
for_each_unit with a BalLds record): for any cumulative weights, grid and
batch size, the waves of all groups take every unit exactly once.  The GPU
side of the same property is tests/test_gpu_slots.py."""
import numpy as np
import pytest

ONE = 1 << 24
GROUPS = 8


def wave_units(n, grid, wpb, cut, block, wib, round_mult=1):
    """The units wave (block, wib) takes: the kernel's loop, restated."""
    g = block % GROUPS
    nwg = (grid - g + GROUPS - 1) // GROUPS * wpb
    lw = (block // GROUPS) * wpb + wib
    nw = grid * wpb
    S = round_mult * nw
    c0, c1 = cut[g], cut[g + 1]
    out = []
    base, lo, k = 0, 0, lw

    def settle():
        nonlocal base, lo, k
        while base < n:
            size = min(n - base, S)
            lo = base + ((size * c0) >> 24)
            hi = base + ((size * c1) >> 24)
            if k < hi - lo:
                return lo + k
            k -= hi - lo
            base += S
        return n

    u = settle()
    while u < n:
        out.append(u)
        k = u - lo + nwg
        u = settle()
    return out


def random_cut(rng):
    w = rng.uniform(1 / 32, 1 / 2, GROUPS)
    w = np.floor(w / w.sum() * ONE).astype(np.int64)
    w[-1] = ONE - w[:-1].sum()
    return np.concatenate([[0], np.cumsum(w)]).tolist()


@pytest.mark.parametrize("seed", range(40))
def test_every_unit_exactly_once(seed):
    rng = np.random.default_rng(seed)
    grid = int(rng.choice([8, 9, 15, 64, 255, 256, 512]))
    wpb = 16
    nw = grid * wpb
    n = int(rng.choice([nw, nw + 1, 2 * nw - 1, 4 * nw, 4 * nw + 7, int(rng.integers(nw, 9 * nw))]))
    cut = random_cut(rng) if seed % 5 else [g * (ONE // GROUPS) for g in range(GROUPS)] + [ONE]
    seen = np.zeros(n, dtype=np.int64)
    rm = int(rng.choice([1, 2]))  # MCK_BAL_ROUND
    for b in range(grid):
        for w in range(wpb):
            for u in wave_units(n, grid, wpb, cut, b, w, round_mult=rm):
                seen[u] += 1
    assert seen.min() == 1 and seen.max() == 1, (grid, n, np.nonzero(seen != 1)[0][:10])


def test_group_shares_follow_the_weights():
    """Group g's share of the units is its weight, to within one unit per
    round, and spread evenly over the group's waves (at most one unit apart)."""
    rng = np.random.default_rng(9)
    grid, wpb = 256, 16
    n = 16384
    cut = random_cut(rng)
    per_group = np.zeros(GROUPS)
    per_wave = [[] for _ in range(GROUPS)]
    for b in range(grid):
        for w in range(wpb):
            k = len(wave_units(n, grid, wpb, cut, b, w))
            per_group[b % GROUPS] += k
            per_wave[b % GROUPS].append(k)
    for g in range(GROUPS):
        assert max(per_wave[g]) - min(per_wave[g]) <= 1, (g, min(per_wave[g]), max(per_wave[g]))
    want = np.diff(np.array(cut, dtype=np.float64)) / ONE * n
    rounds = n // (grid * wpb)
    assert np.all(np.abs(per_group - want) <= rounds + 1), (per_group, want)
