"""Mismatch counts of the verify entry points when MANY payloads fail.

The kernels count mismatches per lane and add them to the caller's counter
once per wave (crc_gpu_device.h, add_mismatches; one atomic per bad payload
made a corrupted buffer ten times slower to verify than a good one), so the
count must stay exact across lanes, waves and workgroups, on the light and the
throughput layouts and through the work queue -- and equal the number of
statuses set.  Two of every three payloads are made to fail."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MSG = 4096  # bytes per message: 16 B core header, 4 B HG header, payload


def _bytes_be32(torch, v):
    v = v.to(torch.int64) & 0xFFFFFFFF
    return torch.stack([(v >> 24) & 0xFF, (v >> 16) & 0xFF, (v >> 8) & 0xFF, v & 0xFF], dim=1).to(torch.uint8)


@pytest.mark.parametrize("n,light", [(1000, None), (1000, "0"), (20000, None), (20000, "1")])
def test_verify_messages_counts_every_bad_message(gpu, n, light, monkeypatch):
    if light is not None:
        monkeypatch.setenv("MCHECKSUM_GPU_LIGHT", light)
    import torch
    t = torch.empty(n * MSG + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, 0xBAD + n)
    pair = np.empty(2 * n, dtype=np.int64)
    pair[0::2] = np.arange(n, dtype=np.int64) * MSG + 20
    pair[1::2] = np.arange(1, n + 1, dtype=np.int64) * MSG
    crc = gpu.checksum_offsets("crc32c", t, torch.from_numpy(pair).cuda())[0::2]
    good = torch.arange(n, device="cuda") % 3 == 0
    # the good messages carry their payload's CRC in the HG header, the others
    # that CRC with one bit flipped
    stored = torch.where(good, crc.to(torch.int64), crc.to(torch.int64) ^ 0x100)
    view = t[:n * MSG].view(n, MSG)
    view[:, 16:20] = _bytes_be32(torch, stored)
    offs = torch.arange(0, (n + 1) * MSG, MSG, dtype=torch.int64, device="cuda")
    status, mism = gpu.verify_messages(t, offs)
    want = (~good).to(torch.uint8)
    assert torch.equal(status, want)
    assert int(mism.item()) == int(want.sum().item())


@pytest.mark.parametrize("method", ["crc32c", "crc64"])
@pytest.mark.parametrize("n", [777, 20000])
def test_verify_offsets_counts_every_mismatch(gpu, method, n):
    import torch
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 9000, size=n)
    off = np.zeros(n + 1, dtype=np.int64)
    off[1:] = np.cumsum(lens)
    t = torch.empty(int(off[-1]) + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, 0x5EED)
    offs = torch.from_numpy(off).cuda()
    crc = gpu.checksum_offsets(method, t, offs)
    flip = torch.arange(n, device="cuda") % 3 != 0
    expected = torch.where(flip, crc ^ 1, crc)
    status, mism = gpu.verify_offsets(method, t, offs, expected)
    assert torch.equal(status, flip.to(torch.uint8))
    assert int(mism.item()) == int(flip.sum().item())


def test_core_header_mismatch_count_equals_statuses(gpu):
    """Random 16-byte headers: (almost) every CRC16 fails; the count must be
    exactly the number of statuses set."""
    import torch
    n = 50000
    t = torch.empty(n * 16 + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, 16)
    offs = torch.arange(0, (n + 1) * 16, 16, dtype=torch.int64, device="cuda")
    status, mism = gpu.verify_core_headers(t, offs, kind="request")
    nbad = int(status.to(torch.int64).sum().item())
    assert nbad > n - 50 and int(mism.item()) == nbad
