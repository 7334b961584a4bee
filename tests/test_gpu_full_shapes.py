"""Every payload of the BASELINE GPU shapes at full size, bit for bit against
the oracle: the headline 65536 x 64 KiB (4 GiB), C3 8192 x 1 MiB CRC-64
(8 GiB), C4 262144 x U[64 B, 64 KiB] offsets (8.6 GB) and C5 2^20 x 64 KiB
(64 GiB, the whole 8-GPU batch on one GPU); plus single payloads past 2 GiB.

The fixed shapes never leave the device: the oracle regenerates the same
splitmix64 payload bytes on the host (oracle_splitmix_batch_fixed, 16
threads).  C4's byte-packed buffer is copied back once.  test_gpu_parity.py
covers the odd shapes and edges at small sizes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_C3 = 0x4D43310000000003
SEED_C4 = 0x4D43310000000004
SEED_C5 = 0x4D43310000000005  # the headline shares C5's seed (bench.py)
THREADS = 16


def _fixed(gpu, method, seed, count, length):
    import torch
    t = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, seed)
    return t, gpu.as_unsigned(gpu.checksum_fixed(method, t, length, count=count)).astype(np.uint64)


def _want_fixed(oracle_mod, method, seed, count, length):
    variant = "sse42" if method == "crc32c" else "table"
    return oracle_mod.splitmix_batch_fixed(method, seed, length, length, 0, count, variant=variant,
                                           nthreads=THREADS)


def _mismatches(got, want):
    bad = np.nonzero(got != want)[0]
    return bad.size, bad[:8].tolist()


def test_headline_every_payload(gpu, oracle_mod):
    t, got = _fixed(gpu, "crc32c", SEED_C5, 65536, 65536)
    del t
    assert _mismatches(got, _want_fixed(oracle_mod, "crc32c", SEED_C5, 65536, 65536)) == (0, [])


def test_c3_every_segment(gpu, oracle_mod):
    t, got = _fixed(gpu, "crc64", SEED_C3, 8192, 1 << 20)
    del t
    assert _mismatches(got, _want_fixed(oracle_mod, "crc64", SEED_C3, 8192, 1 << 20)) == (0, [])


def test_c4_every_payload(gpu, oracle_mod):
    import torch
    count = 262144
    off = oracle_mod.varlen_offsets(SEED_C4, count)
    t = torch.empty(int(off[-1]) + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, SEED_C4)
    offs = torch.from_numpy(off.astype(np.int64)).cuda()
    got = gpu.as_unsigned(gpu.checksum_offsets("crc32c", t, offs, offsets_host=off)).astype(np.uint64)
    host = t[:int(off[-1])].cpu().numpy()
    del t
    want = oracle_mod.batch_offsets("crc32c", host, off, variant="sse42", nthreads=THREADS)
    assert _mismatches(got, want) == (0, [])


def test_c5_on_one_gpu_every_payload_and_split_calls(gpu, oracle_mod):
    """2^20 payloads in one call (the largest single-GPU batch), and the same
    bytes as two calls of 2^19 payloads each."""
    count, length = 1 << 20, 65536
    t, got = _fixed(gpu, "crc32c", SEED_C5, count, length)
    half = count // 2
    lo = gpu.as_unsigned(gpu.checksum_fixed("crc32c", t[:half * length + 64], length, count=half))
    hi = gpu.as_unsigned(gpu.checksum_fixed("crc32c", t[half * length:], length, count=half))
    del t
    assert np.array_equal(np.concatenate([lo, hi]).astype(np.uint64), got)
    assert _mismatches(got, _want_fixed(oracle_mod, "crc32c", SEED_C5, count, length)) == (0, [])


@pytest.mark.parametrize("method", ["crc32c", "crc64"])
def test_payloads_past_2_gib(gpu, oracle_mod, method):
    """Single payloads of more than 2^31 bytes: a fixed batch of one (generic
    and aligned window) and an offsets batch whose middle payload is > 2 GiB
    (the offsets kernel's 64-bit-length path), next to small neighbours."""
    import torch
    big = (1 << 31) + 4096 * 3 + 5
    t = torch.empty(big + (1 << 20) + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, 0xB16)
    host = t[:big + (1 << 20)].cpu().numpy()
    variant = "sse42" if method == "crc32c" else "table"
    for n in (big, (1 << 31) + (1 << 20)):  # ragged length / whole 4 KiB-ring steps
        got = int(gpu.as_unsigned(gpu.checksum_fixed(method, t, n, count=1))[0])
        assert got == oracle_mod.crc(method, host[:n], variant=variant), n
    off = np.array([0, 100, 100 + big, 100 + big + 4097, 100 + big + 4097 + 3], dtype=np.uint64)
    got = gpu.as_unsigned(gpu.checksum_offsets(method, t, torch.from_numpy(off.astype(np.int64)).cuda(),
                                               offsets_host=off)).tolist()
    want = [oracle_mod.crc(method, host[int(off[i]):int(off[i + 1])], variant=variant) for i in range(4)]
    assert got == want
