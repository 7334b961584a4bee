"""Seeded cross-entry-point fuzz of the batch kernels against the oracle.

Each case draws a catalogue model (every 32/64-bit variant the GPU path
serves, MSB-first CRC-64/ECMA-182 included: DESIGN.md sec. 9), an entry point
(fixed-stride, offsets table, verify with planted mismatches, scatter-gather
segments) and a shape -- counts, lengths (0 and past 64 KiB included), strides
and start offsets at every alignment -- plus the layout knobs the host picks
from the batch size (light vs throughput layout, non-temporal loads), so one
run crosses the kernels' dispatch table far from the hand-picked shapes of
test_gpu_parity.py.  Every value is compared with the oracle
(oracle/crc_oracle.c table path, itself pinned to the catalogue check values
and RFC 3720 in test_oracle.py): bit-exact, the integer parity bar.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

METHODS = ["crc32c", "crc32", "crc64", "crc64-ecma182", "crc64-go-iso", "crc64-jones"]
CASES = 120


def _lengths(rng, n, cap):
    kind = rng.integers(0, 4)
    if kind == 0:  # small, zeros included
        return rng.integers(0, 64, n)
    if kind == 1:  # around 1 KiB steps and the 128-B grid
        return rng.choice([0, 1, 15, 16, 17, 127, 128, 129, 1023, 1024, 1025, 2047, 2048, 4095, 4096], n)
    if kind == 2:  # C4's mix
        return rng.integers(64, 65537, n)
    return rng.integers(0, cap, n)  # anything up to cap


@pytest.mark.parametrize("case", range(CASES))
def test_fuzz_case(gpu, oracle_mod, monkeypatch, case):
    import torch
    O = oracle_mod
    rng = np.random.default_rng(0xF022 + 7919 * case)
    method = METHODS[case % len(METHODS)]
    entry = ["fixed", "offsets", "verify", "segments"][rng.integers(0, 4)]
    for var in ("MCHECKSUM_GPU_LIGHT", "MCHECKSUM_GPU_NT"):
        choice = rng.integers(0, 3)  # the size-based default, or forced off / on
        if choice:
            monkeypatch.setenv(var, "1" if choice == 2 else "0")
    lead = int(rng.integers(0, 16))  # start offset of the batch inside its allocation
    if entry == "fixed":
        count = int(rng.integers(1, 3000))
        length = int(rng.choice([int(rng.integers(0, 70000)), 4096, 65536, 1024, 16384, 100]))
        stride = length + int(rng.choice([0, 0, 1, 16, int(rng.integers(0, 300))]))
        nbytes = lead + (count - 1) * stride + length
        if nbytes > (96 << 20):
            count = max(1, ((96 << 20) - lead - length) // max(stride, 1))
            nbytes = lead + (count - 1) * stride + length
        host = O.splitmix_bytes(nbytes, case)
        dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
        got = gpu.as_unsigned(gpu.checksum_fixed(method, dev[lead:], length, count=count, stride=stride))
        want = O.batch_fixed(method, host[lead:], stride, length, count, nthreads=8)
        assert np.array_equal(got.astype(np.uint64), want), (method, count, length, stride, lead)
        return
    if entry in ("offsets", "verify"):
        count = int(rng.integers(1, 5000))
        lens = _lengths(rng, count, 140000).astype(np.uint64)
        off = np.zeros(count + 1, dtype=np.uint64)
        np.cumsum(lens, out=off[1:])
        off += np.uint64(lead)
        host = O.splitmix_bytes(int(off[-1]), case)
        dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
        offs = torch.from_numpy(off.astype(np.int64)).cuda()
        want = O.batch_offsets(method, host, off, nthreads=8)
        if entry == "offsets":
            got = gpu.as_unsigned(gpu.checksum_offsets(method, dev, offs, offsets_host=off))
            assert np.array_equal(got.astype(np.uint64), want), (method, count, lead)
            return
        bad = np.unique(rng.integers(0, count, max(1, count // 50)))
        exp = want.copy()
        exp[bad] ^= np.uint64(1) << np.uint64(int(rng.integers(0, 32)))
        width = 64 if gpu.out_dtype(method) == torch.int64 else 32
        exp_t = torch.from_numpy(exp.astype(np.uint64).view(np.int64) if width == 64
                                 else exp.astype(np.uint32).view(np.int32)).cuda()
        status, mism = gpu.verify_offsets(method, dev, offs, exp_t, offsets_host=off)
        assert sorted(np.nonzero(status.cpu().numpy())[0].tolist()) == bad.tolist(), (method, count)
        assert int(mism.item()) == len(bad)
        return
    # segments: objects of 0..6 segments, each a slice of one buffer at any offset
    nobj = int(rng.integers(1, 600))
    per = rng.integers(0, 7, nobj)
    nseg = int(per.sum())
    seg_len = _lengths(rng, max(nseg, 1), 300000)[:nseg].astype(np.int64)
    pool = O.splitmix_bytes(int(seg_len.sum()) + 4096 * max(nseg, 1) + 64, case)
    dev = torch.from_numpy(pool).cuda()
    starts = rng.integers(0, 4096, max(nseg, 1))[:nseg] + np.concatenate([[0], np.cumsum(seg_len + 4096)[:-1]]) \
        if nseg else np.zeros(0, dtype=np.int64)
    segs = [dev[int(s):int(s) + int(n)] for s, n in zip(starts, seg_len)]
    first = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
    batch = gpu.SegmentBatch(segs, first)
    got = gpu.as_unsigned(batch.checksum(method))
    for j in range(nobj):
        parts = [pool[int(starts[k]):int(starts[k]) + int(seg_len[k])] for k in range(first[j], first[j + 1])]
        w = O.crc(method, np.concatenate(parts) if parts else np.zeros(0, np.uint8))
        assert int(got[j]) == w, (method, j, [int(seg_len[k]) for k in range(first[j], first[j + 1])])
