"""The bench's numpy layout generator equals the oracle's C generator."""
import numpy as np

from mercury_amd import workload as W


def test_varlen_offsets_match_oracle(oracle_mod):
    for seed, n in ((0x4D43310000000004, 262144), (0x4D43310000000004 ^ 1, 1000), (7, 1), (0, 0)):
        got = W.varlen_offsets(seed, n)
        want = oracle_mod.varlen_offsets(seed, n)
        assert got.dtype == np.uint64 and np.array_equal(got, want)
    lens = np.diff(W.varlen_offsets(123, 50000).astype(np.int64))
    assert lens.min() >= 64 and lens.max() <= 65536


def test_splitmix_matches_oracle(oracle_mod):
    xs = [0, 1, 2**63, 2**64 - 1, 0x4D43310000000005]
    assert [int(v) for v in W.splitmix64(np.array(xs, dtype=np.uint64))] == [oracle_mod.splitmix64(x) for x in xs]
