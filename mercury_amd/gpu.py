"""Batch checksums of device-resident payloads on MI355X (include/mchecksum_gpu.h).

Thin torch-facing wrappers over the C ABI: torch only provides device memory
and streams here.  Every function checks tensor shapes, dtypes and bounds on
the host before the kernel launch and raises on any error -- there is no CPU
fallback.  Offsets tables live on the device: they are bounds-checked when a
host copy is passed (offsets_host=...), otherwise trusted, as in the C ABI.
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


def _stream_handle(stream, device=None) -> int:
    """hipStream_t for a call on `device` (the data tensor's device): None =
    that device's current stream; a torch stream must belong to it."""
    if stream is None:
        return torch.cuda.current_stream(device).cuda_stream
    if hasattr(stream, "cuda_stream"):
        if device is not None and getattr(stream, "device", device) != device:
            raise GpuChecksumError(f"stream belongs to {stream.device}, data to {device}")
        return stream.cuda_stream
    return int(stream)


def _same_device(data: torch.Tensor, **tensors):
    """Every tensor argument must live on data's device: the library launches
    on the current device, which _on(data) makes data's."""
    for name, t in tensors.items():
        if t is not None and (not isinstance(t, torch.Tensor) or t.device != data.device):
            raise GpuChecksumError(f"{name} must be a tensor on {data.device}")


def _on(data: torch.Tensor):
    """Make data's device current for the call (the C library picks its table
    pack and queue slot from hipGetDevice())."""
    return torch.cuda.device(data.device)


def _check_device_u8(t: torch.Tensor, name: str):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise GpuChecksumError(f"{name} must be a device (cuda/hip) tensor")
    if not t.is_contiguous():
        raise GpuChecksumError(f"{name} must be contiguous")


def gpu_available() -> bool:
    return bool(_lib().mchecksum_gpu_available())


def queue_faults() -> int:
    """Work-queue protocol faults the batch kernels counted on the current
    device since load (bounded waits that gave up; 0 when healthy).
    Synchronizes the device."""
    return int(_lib().mchecksum_gpu_queue_faults())


QSTAT_KEYS = ("slot", "noslot", "reaped", "busy_skip", "in_flight")


def queue_stats() -> dict:
    """Work-queue slot bookkeeping of the current device (mchecksum_gpu_queue_stats):
    launches given a slot, launches without one (graph captures, no idle slot),
    slots reaped back into the idle pool, busy in-flight slots looked at while
    reaping, slots handed out and not yet reaped."""
    import ctypes
    buf = (ctypes.c_longlong * len(QSTAT_KEYS))()
    rc = _lib().mchecksum_gpu_queue_stats(buf, len(QSTAT_KEYS))
    if rc:
        _err(rc, "queue_stats")
    return dict(zip(QSTAT_KEYS, (int(v) for v in buf)))


def set_error_word(word: torch.Tensor | None) -> None:
    """Fail-closed report (mchecksum_gpu_set_error_word): every later batch call
    of this host thread adds 1 to `word` (a one-element device int32 tensor the
    caller zeroes) when its launch could not hash every payload.  None turns
    the report off.  Keep the tensor alive while it is set."""
    if word is not None and (word.dtype != torch.int32 or not word.is_cuda or word.numel() < 1):
        raise GpuChecksumError("error word must be a device int32 tensor")
    _lib().mchecksum_gpu_set_error_word(word.data_ptr() if word is not None else None)


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
    elif out.numel() < count or out.dtype != out_dtype(method) or not out.is_cuda or not out.is_contiguous():
        raise GpuChecksumError("out tensor has the wrong size, dtype or device, or is not contiguous")
    _same_device(data, out=out)
    with _on(data):
        rc = _lib().mchecksum_gpu_checksum_fixed(method.encode(), data.data_ptr(), stride, length, count,
                                                 out.data_ptr(), _stream_handle(stream, data.device))
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
    elif out.numel() < count or out.dtype != out_dtype(method) or not out.is_cuda or not out.is_contiguous():
        raise GpuChecksumError("out tensor has the wrong size, dtype or device, or is not contiguous")
    _same_device(data, offsets=offsets, out=out)
    with _on(data):
        rc = _lib().mchecksum_gpu_checksum_offsets(method.encode(), data.data_ptr(), offsets.data_ptr(), count,
                                                   out.data_ptr(), _stream_handle(stream, data.device))
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
    _same_device(data, offsets=offsets, expected=expected)
    # status starts "failed": only a hashed payload's verdict overwrites it
    status = torch.ones(count, dtype=torch.uint8, device=data.device)
    mism = torch.zeros(1, dtype=torch.int32, device=data.device)
    with _on(data):
        rc = _lib().mchecksum_gpu_verify_offsets(method.encode(), data.data_ptr(), offsets.data_ptr(), count,
                                                 expected.data_ptr(), status.data_ptr(), mism.data_ptr(),
                                                 _stream_handle(stream, data.device))
    if rc != 0:
        _err(rc, "mchecksum_gpu_verify_offsets")
    return status, mism


def verify_messages(data: torch.Tensor, msg_offsets: torch.Tensor, payload_offset: int = 20, hash_offset: int = 16,
                    method: str = "crc32c", stream=None, offsets_host=None, status=None, mismatches=None):
    """Verify received RPC messages in place: payload after payload_offset,
    expected CRC = network-order u32 at hash_offset (Mercury: 16 B core header,
    4 B HG header).  Returns (status uint8 per message: 1 = fails, count).
    Pass preallocated `status` (uint8, >= count) and `mismatches` (int32, one
    element, zeroed by the caller; the call adds to it) to reuse buffers."""
    _check_device_u8(data, "data")
    _check_offsets(data, msg_offsets, offsets_host)
    count = msg_offsets.numel() - 1
    if status is None:
        status = torch.ones(max(count, 0), dtype=torch.uint8, device=data.device)
    elif status.dtype != torch.uint8 or status.numel() < count or not status.is_cuda:
        raise GpuChecksumError("status must be a device uint8 tensor of at least count elements")
    mism = torch.zeros(1, dtype=torch.int32, device=data.device) if mismatches is None else mismatches
    if mism.dtype != torch.int32 or not mism.is_cuda:
        raise GpuChecksumError("mismatches must be a device int32 tensor")
    _same_device(data, msg_offsets=msg_offsets, status=status, mismatches=mism)
    with _on(data):
        rc = _lib().mchecksum_gpu_verify_messages(method.encode(), data.data_ptr(), msg_offsets.data_ptr(), count,
                                                  payload_offset, hash_offset, status.data_ptr(), mism.data_ptr(),
                                                  _stream_handle(stream, data.device))
    if rc != 0:
        _err(rc, "mchecksum_gpu_verify_messages")
    return status, mism


def _torch_owned(stream, handle: int, device) -> bool:
    """Whether `handle` (the hipStream_t a call ran on, given `stream` as passed)
    is a stream torch created and never destroys: a torch.cuda.Stream from its
    pool (not an ExternalStream wrapping a caller's handle) or the device's
    default stream.  With stream=None the current stream may wrap an external
    handle, which torch cannot tell apart here, so only the default stream
    counts."""
    if stream is None:
        return handle == torch.cuda.default_stream(device).cuda_stream
    return type(stream) is torch.cuda.Stream


class SegmentBatch:
    """A scatter-gather batch prepared once: object j = the concatenation of
    segments[obj_first[j]:obj_first[j+1]] (default: one object), each segment a
    contiguous 1-D uint8 device tensor (views of larger buffers are fine) --
    the bulk-handle shape, HG_Bulk_create's (buf_ptrs, buf_sizes) in device
    memory.  The segment table and the scan workspace stay on the device, so
    `checksum` is one C-ABI call (no host work per launch).  Keep the segment
    tensors alive while the batch is in use.  Calls share the one workspace,
    so a call on another stream than the previous call's first waits for it
    (the C ABI requires a workspace per concurrent call)."""

    def __init__(self, segments, obj_first=None, device=None):
        import numpy as np
        addr, lens, dev = [], [], device
        for t in segments:
            _check_device_u8(t, "segment")
            if t.dim() != 1:
                raise GpuChecksumError("segments must be 1-D byte tensors")
            dev = t.device if dev is None else dev
            if t.device != dev:
                raise GpuChecksumError("segments must share one device")
            addr.append(t.data_ptr())
            lens.append(t.numel())
        self.nseg = len(addr)
        first = np.asarray([0, self.nseg] if obj_first is None else obj_first, dtype=np.int64)
        if first.ndim != 1 or len(first) < 1 or np.any(first[1:] < first[:-1]) or first[0] < 0 \
                or first[-1] > self.nseg:
            raise GpuChecksumError("obj_first must be non-decreasing indices into segments")
        self.nobj = len(first) - 1
        self.device = dev if dev is not None else torch.device("cuda", torch.cuda.current_device())
        self.bytes = int(np.sum(np.asarray(lens, dtype=np.int64)[first[0]:first[-1]])) if self.nseg else 0
        self.meta = torch.from_numpy(np.concatenate([np.asarray(addr, dtype=np.uint64).view(np.int64),
                                                     np.asarray(lens, dtype=np.int64), first])).to(self.device)
        self.work = torch.empty((_lib().mchecksum_gpu_segments_work_size(self.nseg) + 7) // 8, dtype=torch.int64,
                                device=self.device)
        self._last = None  # (stream handle, its torch stream, event after the call or None) of the last call

    def checksum(self, method: str, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        if out is None:
            out = torch.empty(self.nobj, dtype=out_dtype(method), device=self.device)
        elif out.numel() < self.nobj or out.dtype != out_dtype(method) or not out.is_cuda or not out.is_contiguous():
            raise GpuChecksumError("out tensor has the wrong size, dtype or device, or is not contiguous")
        if out.device != self.device:
            raise GpuChecksumError(f"out must be on {self.device}")
        base, n = self.meta.data_ptr(), self.nseg
        with torch.cuda.device(self.device):
            h = _stream_handle(stream, self.device)
            # (graph capture: replays are ordered by the graph's user; no events)
            track = not torch.cuda.is_current_stream_capturing()
            s = (torch.cuda.ExternalStream(h) if h else torch.cuda.default_stream(self.device)) if track else None
            if track and self._last is not None and self._last[0] != h:
                # the workspace is still the previous call's: this stream waits
                # for it.  On a stream torch owns (its pool's or the default
                # stream: never destroyed) the event is recorded now, at the
                # switch, after everything queued so far -- not after every
                # call (a marker packet between the kernels costs ~3 us); any
                # other stream (a raw handle, a torch.cuda.ExternalStream, or
                # a current stream that may be one) may be destroyed by then,
                # so its event was recorded right after the call.
                ev = self._last[2]
                if ev is None:
                    ev = torch.cuda.Event()
                    ev.record(self._last[1])
                s.wait_event(ev)
            rc = _lib().mchecksum_gpu_checksum_segments(method.encode(), base, base + 8 * n, n, base + 16 * n,
                                                        self.nobj, self.work.data_ptr(), self.work.numel() * 8,
                                                        out.data_ptr(), h)
            if rc == 0 and track:
                ev = None
                if not _torch_owned(stream, h, self.device):
                    ev = torch.cuda.Event()
                    ev.record(s)
                self._last = (h, s, ev)
        if rc != 0:
            _err(rc, "mchecksum_gpu_checksum_segments")
        return out


def checksum_segments(method: str, segments, obj_first=None, out: torch.Tensor | None = None,
                      stream=None) -> torch.Tensor:
    """One-shot SegmentBatch(segments, obj_first).checksum(method)."""
    b = SegmentBatch(segments, obj_first)
    out = b.checksum(method, out, stream)
    # the batch's device table and workspace are freed on return: the caching
    # allocator orders their reuse after this launch on the current stream;
    # another stream must be recorded
    if stream is not None:
        if isinstance(stream, torch.cuda.Stream):
            b.meta.record_stream(stream)
            b.work.record_stream(stream)
        else:
            torch.cuda.synchronize(b.device)
    return out


def verify_core_headers(data: torch.Tensor, msg_offsets: torch.Tensor, kind: str = "request",
                        method: str = "crc16", stream=None, offsets_host=None):
    """Check the CRC16 of each message's 16-byte Mercury core header
    (kind "request" or "response").  Returns (status uint8 per message, count)."""
    from ._lib import CORE_HEADER_REQUEST, CORE_HEADER_RESPONSE
    k = {"request": CORE_HEADER_REQUEST, "response": CORE_HEADER_RESPONSE}.get(kind)
    if k is None:
        raise GpuChecksumError("kind must be 'request' or 'response'")
    _check_device_u8(data, "data")
    _check_offsets(data, msg_offsets, offsets_host)
    count = msg_offsets.numel() - 1
    _same_device(data, msg_offsets=msg_offsets)
    status = torch.ones(max(count, 0), dtype=torch.uint8, device=data.device)
    mism = torch.zeros(1, dtype=torch.int32, device=data.device)
    with _on(data):
        rc = _lib().mchecksum_gpu_verify_core_headers(method.encode(), k, data.data_ptr(), msg_offsets.data_ptr(),
                                                      count, status.data_ptr(), mism.data_ptr(),
                                                      _stream_handle(stream, data.device))
    if rc != 0:
        _err(rc, "mchecksum_gpu_verify_core_headers")
    return status, mism


XDR_INT, XDR_OPAQUE, XDR_OPAQUE_LEN, XDR_RAW, XDR_RAW_LEN, XDR_SKIP_IF_ZERO = 0, 1, 2, 3, 4, 5


def checksum_xdr(method: str, data: torch.Tensor, msg_offsets: torch.Tensor, schema, status: bool = False,
                 stream=None, offsets_host=None, out: torch.Tensor | None = None):
    """Proc checksum of messages serialized in XDR mode (include/mchecksum_gpu.h,
    mchecksum_gpu_checksum_xdr): schema = [(kind, size), ...] with the XDR_*
    kinds.  Returns the CRC tensor, or (CRCs, status) with status=True
    (status 1 = the schema runs past the message)."""
    from ._lib import XdrField
    _check_device_u8(data, "data")
    _check_offsets(data, msg_offsets, offsets_host)
    _same_device(data, msg_offsets=msg_offsets)
    count = msg_offsets.numel() - 1
    fields = (XdrField * max(1, len(schema)))(*[XdrField(int(k), int(z)) for k, z in schema])
    if out is None:
        out = torch.empty(max(count, 0), dtype=out_dtype(method), device=data.device)
    elif (out.numel() < count or out.dtype != out_dtype(method) or out.device != data.device
          or not out.is_contiguous()):
        raise GpuChecksumError("out tensor has the wrong size, dtype or device, or is not contiguous")
    st = torch.ones(max(count, 0), dtype=torch.uint8, device=data.device) if status else None
    with _on(data):
        rc = _lib().mchecksum_gpu_checksum_xdr(method.encode(), fields, len(schema), data.data_ptr(),
                                               msg_offsets.data_ptr(), count, out.data_ptr(),
                                               st.data_ptr() if st is not None else None,
                                               _stream_handle(stream, data.device))
    if rc != 0:
        _err(rc, "mchecksum_gpu_checksum_xdr")
    return (out, st) if status else out


def fill_splitmix(t: torch.Tensor, seed: int, first_word: int = 0, stream=None) -> torch.Tensor:
    """Fill a device tensor with the synthetic payload bytes of SURVEY.md 8(d)."""
    _check_device_u8(t, "tensor")
    if t.data_ptr() % 16:
        raise GpuChecksumError("tensor must be 16-byte aligned")
    B = load_bench_library()
    with _on(t):
        rc = B.mck_bench_fill_splitmix(t.data_ptr(), t.numel() * t.element_size(), seed & (2**64 - 1),
                                       first_word, _stream_handle(stream, t.device))
    if rc != 0:
        raise GpuChecksumError(f"fill_splitmix failed rc={rc}")
    return t


class HostGate:
    """Test utility (libmchecksum_bench.so): a kernel that holds a stream until
    the host calls release() -- one wave polling a word of coherent host
    memory -- or until max_seconds pass, which `expired` then reports.  Used
    to keep launches queued for exactly as long as a test needs."""

    def __init__(self):
        self._B = load_bench_library()
        self._mem = self._B.mck_bench_host_alloc(8)
        if not self._mem:
            raise GpuChecksumError("hipHostMalloc failed")
        self._flag = ctypes.c_uint32.from_address(self._mem)
        self._exp = ctypes.c_uint32.from_address(self._mem + 4)

    def hold(self, stream, max_seconds: float = 20.0) -> None:
        self._flag.value = 0
        self._exp.value = 0
        h = _stream_handle(stream)
        if self._B.mck_bench_gate(self._mem, self._mem + 4, float(max_seconds), h) != 0:
            raise GpuChecksumError("gate launch failed")

    def release(self) -> None:
        self._flag.value = 1

    @property
    def expired(self) -> bool:
        return bool(self._exp.value)

    def close(self) -> None:
        if self._mem:
            self.release()
            torch.cuda.synchronize()
            self._B.mck_bench_host_free(self._mem)
            self._mem = None


def as_unsigned(x: torch.Tensor):
    """Device CRC tensor -> numpy unsigned array on the host."""
    import numpy as np
    a = x.detach().cpu().numpy()
    return a.view(np.uint32 if a.dtype == np.int32 else np.uint64)
