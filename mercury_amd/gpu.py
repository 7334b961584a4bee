"""Batch checksums of device-resident payloads on MI355X (include/mchecksum_gpu.h).

Thin torch-facing wrappers over the C ABI: torch only provides device memory
and streams here.  Every function checks shapes on the host before the
kernel launch (so a bad argument can never turn into an out-of-bounds read on
the GPU) and raises on any error -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import load_bench_library, load_library

_WIDTH = {"crc32c": 4, "crc32": 4, "crc64": 8}


class GpuChecksumError(RuntimeError):
    pass


def _lib():
    return load_library()


def _err(rc: int, what: str):
    msg = _lib().mchecksum_gpu_last_error()
    raise GpuChecksumError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def out_dtype(method: str) -> torch.dtype:
    w = _WIDTH.get(method, 8 if method.startswith("crc64") else 4)
    return torch.int32 if w == 4 else torch.int64


def _stream_handle(stream) -> int:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return int(stream)


def _check_device_u8(t: torch.Tensor, name: str):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise GpuChecksumError(f"{name} must be a device (cuda/hip) tensor")
    if not t.is_contiguous():
        raise GpuChecksumError(f"{name} must be contiguous")


def gpu_available() -> bool:
    return bool(_lib().mchecksum_gpu_available())


def prepare(method: str = "crc32c") -> None:
    rc = _lib().mchecksum_gpu_prepare(method.encode())
    if rc != 0:
        _err(rc, f"mchecksum_gpu_prepare({method})")


def lanes_per_payload(method: str, length: int) -> int:
    return int(_lib().mchecksum_gpu_lanes_per_payload(method.encode(), length))


def checksum_fixed(method: str, data: torch.Tensor, length: int, count: int | None = None,
                   stride: int | None = None, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """CRC of payload i = data[i*stride : i*stride+length] for i < count.

    Returns a device tensor (int32 for crc32c, int64 for crc64) holding the
    host-order CRC values (reinterpret as unsigned)."""
    _check_device_u8(data, "data")
    nbytes = data.numel() * data.element_size()
    stride = length if stride is None else stride
    if count is None:
        count = nbytes // stride if stride else 0
    if count and (count - 1) * stride + length > nbytes:
        raise GpuChecksumError("batch extends past the end of data")
    if count > 1 and stride < length:
        raise GpuChecksumError("stride smaller than length")
    if out is None:
        out = torch.empty(count, dtype=out_dtype(method), device=data.device)
    elif out.numel() < count or out.dtype != out_dtype(method) or not out.is_cuda:
        raise GpuChecksumError("out tensor has the wrong size, dtype or device")
    rc = _lib().mchecksum_gpu_checksum_fixed(method.encode(), data.data_ptr(), stride, length, count,
                                             out.data_ptr(), _stream_handle(stream))
    if rc != 0:
        _err(rc, "mchecksum_gpu_checksum_fixed")
    return out


def _check_offsets(data, offsets, offsets_host):
    if offsets.dtype != torch.int64 or not offsets.is_cuda or not offsets.is_contiguous():
        raise GpuChecksumError("offsets must be a contiguous device int64 tensor")
    if offsets_host is not None:
        import numpy as np
        oh = np.asarray(offsets_host, dtype=np.uint64)
        if len(oh) != offsets.numel():
            raise GpuChecksumError("offsets_host does not match offsets")
        if len(oh) > 1 and (np.any(oh[1:] < oh[:-1])):
            raise GpuChecksumError("offsets must be non-decreasing")
        if len(oh) and int(oh[-1]) > data.numel() * data.element_size():
            raise GpuChecksumError("offsets extend past the end of data")


def checksum_offsets(method: str, data: torch.Tensor, offsets: torch.Tensor, out: torch.Tensor | None = None,
                     stream=None, offsets_host=None) -> torch.Tensor:
    """CRC of payload i = data[offsets[i] : offsets[i+1]] (offsets: count+1 int64).

    Pass offsets_host (a host copy) to have the table validated before launch."""
    _check_device_u8(data, "data")
    _check_offsets(data, offsets, offsets_host)
    count = offsets.numel() - 1
    if count < 0:
        raise GpuChecksumError("offsets needs at least one entry")
    if out is None:
        out = torch.empty(count, dtype=out_dtype(method), device=data.device)
    rc = _lib().mchecksum_gpu_checksum_offsets(method.encode(), data.data_ptr(), offsets.data_ptr(), count,
                                               out.data_ptr(), _stream_handle(stream))
    if rc != 0:
        _err(rc, "mchecksum_gpu_checksum_offsets")
    return out


def verify_offsets(method: str, data: torch.Tensor, offsets: torch.Tensor, expected: torch.Tensor,
                   stream=None, offsets_host=None):
    """Returns (status uint8 per payload: 1 = mismatch, mismatch count tensor)."""
    _check_device_u8(data, "data")
    _check_offsets(data, offsets, offsets_host)
    count = offsets.numel() - 1
    if expected.numel() < count or expected.dtype != out_dtype(method) or not expected.is_cuda:
        raise GpuChecksumError("expected has the wrong size, dtype or device")
    status = torch.empty(count, dtype=torch.uint8, device=data.device)
    mism = torch.zeros(1, dtype=torch.int32, device=data.device)
    rc = _lib().mchecksum_gpu_verify_offsets(method.encode(), data.data_ptr(), offsets.data_ptr(), count,
                                             expected.data_ptr(), status.data_ptr(), mism.data_ptr(),
                                             _stream_handle(stream))
    if rc != 0:
        _err(rc, "mchecksum_gpu_verify_offsets")
    return status, mism


def verify_messages(data: torch.Tensor, msg_offsets: torch.Tensor, payload_offset: int = 20, hash_offset: int = 16,
                    method: str = "crc32c", stream=None, offsets_host=None):
    """Verify received RPC messages in place: payload after payload_offset,
    expected CRC = network-order u32 at hash_offset (Mercury: 16 B core header,
    4 B HG header).  Returns (status uint8 per message: 1 = fails, count)."""
    _check_device_u8(data, "data")
    _check_offsets(data, msg_offsets, offsets_host)
    count = msg_offsets.numel() - 1
    status = torch.empty(max(count, 0), dtype=torch.uint8, device=data.device)
    mism = torch.zeros(1, dtype=torch.int32, device=data.device)
    rc = _lib().mchecksum_gpu_verify_messages(method.encode(), data.data_ptr(), msg_offsets.data_ptr(), count,
                                              payload_offset, hash_offset, status.data_ptr(), mism.data_ptr(),
                                              _stream_handle(stream))
    if rc != 0:
        _err(rc, "mchecksum_gpu_verify_messages")
    return status, mism


def fill_splitmix(t: torch.Tensor, seed: int, first_word: int = 0, stream=None) -> torch.Tensor:
    """Fill a device tensor with the synthetic payload bytes of SURVEY.md 8(d)."""
    _check_device_u8(t, "tensor")
    if t.data_ptr() % 16:
        raise GpuChecksumError("tensor must be 16-byte aligned")
    B = load_bench_library()
    rc = B.mck_bench_fill_splitmix(t.data_ptr(), t.numel() * t.element_size(), seed & (2**64 - 1),
                                   first_word, _stream_handle(stream))
    if rc != 0:
        raise GpuChecksumError(f"fill_splitmix failed rc={rc}")
    return t


def as_unsigned(x: torch.Tensor):
    """Device CRC tensor -> numpy unsigned array on the host."""
    import numpy as np
    a = x.detach().cpu().numpy()
    return a.view(np.uint32 if a.dtype == np.int32 else np.uint64)
