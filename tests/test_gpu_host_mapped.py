"""Batch entry points on HOST memory mapped into the GPU's address space.

SURVEY.md 8(f)1 asks for batched verify "straight from NA multi-recv
buffers": Mercury's multi-recv buffers are host allocations made once per
context (/root/reference/src/mercury_core.c:2092-2132, sliced per message at
:4667-4714).  Registered once with hipHostRegister(..., Mapped), their device
alias (hipHostGetDevicePointer) is a valid `dev_base` for the mchecksum_gpu_*
entry points (include/mchecksum_gpu.h: "any device-accessible allocation"):
the kernels then read the payload bytes over PCIe with no staging copy.  The
same holds for hipHostMalloc memory.  These tests call the C ABI directly on
such aliases (offsets table and outputs in device memory) and compare every
value with the oracle; tools/zero_copy.py measures the rate.
"""
import ctypes
import mmap
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REGISTER_MAPPED = 0x2  # hipHostRegisterMapped


@pytest.fixture(scope="module")
def hip():
    import torch
    L = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    vp = ctypes.c_void_p
    L.hipHostRegister.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint]
    L.hipHostUnregister.argtypes = [vp]
    L.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_uint]
    L.hipHostMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
    L.hipHostFree.argtypes = [vp]
    return L


class _Registered:
    """A malloc-like (mmap) host buffer registered with the GPU, as an NA
    plugin's receive buffer would be; .host is a numpy view, .dev the alias."""

    def __init__(self, hip, nbytes):
        self.hip, self.n = hip, nbytes
        self.mm = mmap.mmap(-1, max(nbytes, 1))
        self.host = np.frombuffer(self.mm, dtype=np.uint8, count=nbytes)
        self.ptr = ctypes.addressof(ctypes.c_char.from_buffer(self.mm))
        assert hip.hipHostRegister(self.ptr, max(nbytes, 1), REGISTER_MAPPED) == 0
        d = ctypes.c_void_p()
        assert hip.hipHostGetDevicePointer(ctypes.byref(d), self.ptr, 0) == 0
        self.dev = d.value

    def close(self):
        assert self.hip.hipHostUnregister(self.ptr) == 0
        del self.host
        self.mm.close()


class _Pinned:
    """hipHostMalloc memory."""

    def __init__(self, hip, nbytes):
        self.hip = hip
        p = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(p), max(nbytes, 1), 0) == 0
        self.ptr = p.value
        self.host = np.ctypeslib.as_array((ctypes.c_uint8 * max(nbytes, 1)).from_address(self.ptr))[:nbytes]
        d = ctypes.c_void_p()
        assert hip.hipHostGetDevicePointer(ctypes.byref(d), self.ptr, 0) == 0
        self.dev = d.value

    def close(self):
        del self.host
        assert self.hip.hipHostFree(self.ptr) == 0


def _batch(oracle_mod, n, seed, lo=64, hi=8192):
    rng = np.random.default_rng(seed)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(rng.integers(lo, hi + 1, n).astype(np.uint64), out=off[1:])
    return off, oracle_mod.splitmix_bytes(int(off[-1]) + 64, seed)


@pytest.mark.parametrize("kind", ["registered", "hipHostMalloc"])
@pytest.mark.parametrize("method", ["crc32c", "crc64"])
def test_checksum_offsets_from_mapped_host_memory(gpu, hip, oracle_mod, kind, method):
    import torch
    off, data = _batch(oracle_mod, 3000, 0x4E41)  # > 1024 payloads: throughput layout, work queue
    buf = (_Registered if kind == "registered" else _Pinned)(hip, len(data))
    try:
        buf.host[:] = data
        offs = torch.from_numpy(off.astype(np.int64)).cuda()
        out = torch.empty(3000, dtype=gpu.out_dtype(method), device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        rc = gpu._lib().mchecksum_gpu_checksum_offsets(method.encode(), buf.dev, offs.data_ptr(), 3000,
                                                      out.data_ptr(), s)
        assert rc == 0
        torch.cuda.synchronize()
        want = oracle_mod.batch_offsets(method, data, off, nthreads=8)
        assert np.array_equal(gpu.as_unsigned(out).astype(np.uint64), want)
    finally:
        buf.close()


def test_verify_messages_in_registered_recv_buffer(gpu, hip, oracle_mod):
    """hg_get_struct's check for a whole multi-recv buffer: messages = 16 B
    core header + 4 B HG header (CRC-32C of the payload, network order) +
    payload, packed back to back in a registered host buffer; two corrupted
    payloads are flagged exactly."""
    import torch
    O = oracle_mod
    n = 2500
    off, data = _batch(O, n, 0x4E42, lo=20, hi=6000)
    data = data.copy()
    for i in range(n):
        a, b = int(off[i]), int(off[i + 1])
        data[a + 16:a + 20] = np.frombuffer(O.crc("crc32c", data[a + 20:b]).to_bytes(4, "big"), dtype=np.uint8)
    bad = [7, 1999]
    for i in bad:
        a, b = int(off[i]), int(off[i + 1])
        data[(a + 20 + b) // 2] ^= 0x40
    buf = _Registered(hip, len(data))
    try:
        buf.host[:] = data
        offs = torch.from_numpy(off.astype(np.int64)).cuda()
        status = torch.ones(n, dtype=torch.uint8, device="cuda")
        mism = torch.zeros(1, dtype=torch.int32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        rc = gpu._lib().mchecksum_gpu_verify_messages(b"crc32c", buf.dev, offs.data_ptr(), n, 20, 16,
                                                      status.data_ptr(), mism.data_ptr(), s)
        assert rc == 0
        torch.cuda.synchronize()
        assert np.nonzero(status.cpu().numpy())[0].tolist() == bad
        assert int(mism.item()) == len(bad)
    finally:
        buf.close()
