"""Split CRC-64 (crc_gpu_device.h, crc64_batch_kernel<..., SPLIT>): large
aligned payloads run as 256 KiB pieces on the work queue.  When every queue
chunk holds whole payloads (SplitPlan::whole) the pieces combine in their
workgroup's LDS and the last one stores the CRC; otherwise -- graph captures,
plans whose chunks cut payloads -- they XOR into an output zeroed by a kernel
first.  Both ways against the oracle (MCHECKSUM_GPU_SPLIT_LDS=0 forces the
second), over plans of each kind.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = 16
SEED = 0x5B17


@pytest.mark.parametrize("count,length", [
    (8192, 1 << 20),     # C3: 32768 pieces, 4 per payload -> combined in the workgroup
    (16384, 512 << 10),  # 2 pieces per payload, 16 payloads per full chunk
    (1024, 2 << 20),     # 8192 pieces: small chunks cut payloads -> zeroed output
    (64, 16 << 20),      # 64 pieces per payload -> zeroed output
])
def test_split_crc64_both_combines(gpu, oracle_mod, monkeypatch, count, length):
    import torch
    t = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, SEED)
    want = oracle_mod.splitmix_batch_fixed("crc64", SEED, length, length, 0, count, variant="table", nthreads=THREADS)
    stale = torch.full((count,), -1, dtype=torch.int64, device="cuda")
    got = gpu.as_unsigned(gpu.checksum_fixed("crc64", t, length, count=count, out=stale)).astype(np.uint64)
    assert np.array_equal(got, want)
    monkeypatch.setenv("MCHECKSUM_GPU_SPLIT_LDS", "0")
    stale.fill_(-1)
    got0 = gpu.as_unsigned(gpu.checksum_fixed("crc64", t, length, count=count, out=stale)).astype(np.uint64)
    assert np.array_equal(got0, want)


def test_split_crc64_back_to_back(gpu, oracle_mod):
    """Launches in flight together on one stream (each its own slot and LDS
    state), then a payload changed: every result exact."""
    import torch
    count, length = 8192, 1 << 20
    t = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, SEED)
    want = oracle_mod.splitmix_batch_fixed("crc64", SEED, length, length, 0, count, variant="table", nthreads=THREADS)
    outs = [gpu.checksum_fixed("crc64", t, length, count=count) for _ in range(6)]
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(gpu.as_unsigned(o).astype(np.uint64), want)
    p = count - 5
    t[p * length + 12345] ^= 0x40
    got = gpu.as_unsigned(gpu.checksum_fixed("crc64", t, length, count=count)).astype(np.uint64)
    host = t[p * length:(p + 1) * length].cpu().numpy()
    assert int(got[p]) == oracle_mod.crc("crc64", host, variant="table")
    assert np.array_equal(np.delete(got, p), np.delete(want, p))
