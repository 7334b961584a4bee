"""Empty batches through every GPU entry point: count 0 (and nseg / nobj 0 for
scatter-gather objects) is a valid call that returns 0, launches nothing that
writes, and leaves the caller's output, status and mismatch words as they were
(Mercury may hand over an empty multi-recv window or a bulk handle without
segments).  Every call goes through the C ABI with real device buffers."""
import pytest

pytestmark = pytest.mark.gpu

SENTINEL = 0x5A


def _bufs(torch):
    out = torch.full((64,), SENTINEL, dtype=torch.uint8, device="cuda")
    status = torch.full((64,), SENTINEL, dtype=torch.uint8, device="cuda")
    mism = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    data = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    offs = torch.zeros(8, dtype=torch.int64, device="cuda")
    return out, status, mism, data, offs


@pytest.mark.parametrize("method", ["crc32c", "crc64"])
def test_empty_batches_touch_nothing(gpu, method):
    import torch
    from mercury_amd._lib import XdrField
    L = gpu._lib()
    out, status, mism, data, offs = _bufs(torch)
    s = torch.cuda.current_stream().cuda_stream
    m = method.encode()
    p = lambda t: t.data_ptr()  # noqa: E731
    assert L.mchecksum_gpu_checksum_fixed(m, p(data), 4096, 4096, 0, p(out), s) == 0
    assert L.mchecksum_gpu_checksum_offsets(m, p(data), p(offs), 0, p(out), s) == 0
    assert L.mchecksum_gpu_verify_offsets(m, p(data), p(offs), 0, p(out), p(status), p(mism), s) == 0
    if method == "crc32c":
        assert L.mchecksum_gpu_verify_messages(m, p(data), p(offs), 0, 20, 16, p(status), p(mism), s) == 0
    work = torch.zeros(max(1, L.mchecksum_gpu_segments_work_size(0)) // 8 + 1, dtype=torch.int64, device="cuda")
    assert L.mchecksum_gpu_checksum_segments(m, p(offs), p(offs), 0, p(offs), 0, p(work), work.numel() * 8,
                                             p(out), s) == 0
    fields = (XdrField * 1)(XdrField(0, 4))
    assert L.mchecksum_gpu_checksum_xdr(m, fields, 1, p(data), p(offs), 0, p(out), p(status), s) == 0
    assert L.mchecksum_gpu_verify_core_headers(b"crc16", 0, p(data), p(offs), 0, p(status), p(mism), s) == 0
    torch.cuda.synchronize()
    assert bool((out == SENTINEL).all()), "an empty batch wrote outputs"
    assert bool((status == SENTINEL).all()), "an empty batch wrote status bytes"
    assert int(mism.item()) == 7, "an empty batch touched the mismatch counter"


def test_empty_batch_with_null_buffers(gpu):
    """count 0 needs no buffers at all (NULL base, offsets and outputs)."""
    L = gpu._lib()
    assert L.mchecksum_gpu_checksum_fixed(b"crc32c", None, 0, 0, 0, None, None) == 0
    assert L.mchecksum_gpu_checksum_offsets(b"crc64", None, None, 0, None, None) == 0
    assert L.mchecksum_gpu_verify_offsets(b"crc32c", None, None, 0, None, None, None, None) == 0
    assert L.mchecksum_gpu_verify_messages(b"crc32c", None, None, 0, 20, 16, None, None, None) == 0
