"""ctypes view of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker -- never by mercury_amd/.
See crc_oracle.h for what is restated and what is pinned (CRC-32C: RFC 3720 +
SSE4.2 hardware; CRC-64 / CRC-16 variants: parity unpinned).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

VARIANT_TABLE, VARIANT_SSE42, VARIANT_BITWISE, VARIANT_SLICE8 = 0, 1, 2, 3


class Model(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char_p),
        ("width", ctypes.c_int),
        ("poly", ctypes.c_uint64),
        ("refin", ctypes.c_int),
        ("refout", ctypes.c_int),
        ("init", ctypes.c_uint64),
        ("xorout", ctypes.c_uint64),
        ("check", ctypes.c_uint64),
    ]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER(Model)
        L.oracle_models.restype = P
        L.oracle_model_by_name.restype = P
        L.oracle_model_by_name.argtypes = [ctypes.c_char_p]
        L.oracle_crc_bitwise.restype = ctypes.c_uint64
        L.oracle_crc_bitwise.argtypes = [P, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_crc_table.restype = ctypes.c_uint64
        L.oracle_crc_table.argtypes = [P, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_crc_slice8.restype = ctypes.c_uint64
        L.oracle_crc_slice8.argtypes = [P, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_crc32c_sse42.restype = ctypes.c_uint32
        L.oracle_crc32c_sse42.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]
        L.oracle_fill_splitmix.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_splitmix64.restype = ctypes.c_uint64
        L.oracle_splitmix64.argtypes = [ctypes.c_uint64]
        L.oracle_varlen_offsets.argtypes = [ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                            ctypes.c_void_p]
        L.oracle_batch_fixed.restype = ctypes.c_int
        L.oracle_batch_fixed.argtypes = [P, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        L.oracle_batch_offsets.restype = ctypes.c_int
        L.oracle_batch_offsets.argtypes = [P, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_void_p, ctypes.c_int]
        L.oracle_splitmix_batch_fixed.restype = ctypes.c_int
        L.oracle_splitmix_batch_fixed.argtypes = [P, ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t,
                                                  ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                                  ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


def model(name: str):
    m = lib().oracle_model_by_name(name.encode())
    if not m:
        raise KeyError(name)
    return m


def models():
    out, p, i = [], lib().oracle_models(), 0
    while p[i].name:
        out.append(p[i])
        i += 1
    return out


def _buf(data):
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data, dtype=np.uint8)
    else:
        a = np.frombuffer(bytes(data), dtype=np.uint8)
    return a, (a.ctypes.data if a.size else None)


def crc(method: str, data, variant: str = "table") -> int:
    a, p = _buf(data)
    m = model(method)
    if variant == "bitwise":
        return int(lib().oracle_crc_bitwise(m, p, a.size))
    if variant == "slice8":
        return int(lib().oracle_crc_slice8(m, p, a.size))
    if variant == "sse42":
        ok = ctypes.c_int(0)
        v = lib().oracle_crc32c_sse42(p, a.size, ctypes.byref(ok))
        if not ok.value:
            raise RuntimeError("no SSE4.2 on this CPU")
        return int(v)
    return int(lib().oracle_crc_table(m, p, a.size))


def splitmix64(x: int) -> int:
    return int(lib().oracle_splitmix64(ctypes.c_uint64(x & (2**64 - 1))))


def splitmix_bytes(nbytes: int, seed: int, first_word: int = 0) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    if nbytes:
        lib().oracle_fill_splitmix(out.ctypes.data, nbytes, seed & (2**64 - 1), first_word)
    return out


def varlen_offsets(seed: int, count: int, min_len: int = 64, max_len: int = 65536) -> np.ndarray:
    off = np.empty(count + 1, dtype=np.uint64)
    lib().oracle_varlen_offsets(seed & (2**64 - 1), count, min_len, max_len, off.ctypes.data)
    return off


_VAR = {"table": VARIANT_TABLE, "sse42": VARIANT_SSE42, "bitwise": VARIANT_BITWISE, "slice8": VARIANT_SLICE8}


def batch_fixed(method, data: np.ndarray, stride: int, length: int, count: int, variant="table", nthreads=1):
    out = np.zeros(count, dtype=np.uint64)
    a, p = _buf(data)
    rc = lib().oracle_batch_fixed(model(method), _VAR[variant], p, stride, length, count,
                                  out.ctypes.data, nthreads)
    if rc:
        raise RuntimeError("oracle_batch_fixed failed")
    return out


def batch_offsets(method, data: np.ndarray, offsets: np.ndarray, variant="table", nthreads=1):
    count = len(offsets) - 1
    out = np.zeros(count, dtype=np.uint64)
    a, p = _buf(data)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    rc = lib().oracle_batch_offsets(model(method), _VAR[variant], p, off.ctypes.data, count,
                                    out.ctypes.data, nthreads)
    if rc:
        raise RuntimeError("oracle_batch_offsets failed")
    return out


def splitmix_batch_fixed(method, seed, stride, length, first, count, variant="table", nthreads=1):
    """CRCs of payloads [first, first+count) of a virtual splitmix buffer
    (payload i = bytes [i*stride, i*stride+length)) without materialising it."""
    out = np.zeros(count, dtype=np.uint64)
    rc = lib().oracle_splitmix_batch_fixed(model(method), _VAR[variant], seed & (2**64 - 1), stride, length,
                                           first, count, out.ctypes.data, nthreads)
    if rc:
        raise RuntimeError("oracle_splitmix_batch_fixed failed")
    return out


# ------------------------------------------------------------------- XDR ----
# CPU restatement of what Mercury's proc layer hashes in XDR mode
# (HG_HAS_XDR; /root/reference/src/mercury_proc.h:110-122 HG_PROC_TYPE,
# :147-160 HG_PROC_BYTES; save/restore_ptr src/mercury_proc.c:277-335): each
# typed field occupies RNDUP(sizeof(type)) big-endian wire bytes (xdr_<type>;
# 1/2/4-byte integers as one 32-bit word, 8-byte ones as two, high first) but
# the checksum is updated with the sizeof(type) bytes of the host variable --
# little-endian on this host; byte arrays are xdr_opaque (bytes + zero pad to
# 4), hashed without the pad; save_ptr regions are raw and exact.  Schema kinds
# as include/mchecksum_gpu.h (MCHECKSUM_XDR_*).
XDR_INT, XDR_OPAQUE, XDR_OPAQUE_LEN, XDR_RAW, XDR_RAW_LEN, XDR_SKIP_IF_ZERO = 0, 1, 2, 3, 4, 5


def xdr_encode(schema, values) -> bytes:
    """XDR wire image of one message: values[i] is the integer (INT) or the
    bytes (OPAQUE*/RAW*) of the i-th non-SKIP field that is present."""
    out, vals, last, f = bytearray(), list(values), None, 0
    while f < len(schema):
        kind, size = schema[f]
        if kind == XDR_SKIP_IF_ZERO:
            if last == 0:
                f += size
            f += 1
            continue
        v = vals.pop(0)
        if kind == XDR_INT:
            slot = 4 if size <= 4 else 8
            # xdr_<type>: the value as a 32-bit (signed types sign-extended)
            # or 64-bit big-endian integer
            out += (int(v) & ((1 << (8 * slot)) - 1)).to_bytes(slot, "big")
            last = int(v) & ((1 << (8 * size)) - 1)
        else:
            b = bytes(v)
            out += b
            if kind in (XDR_OPAQUE, XDR_OPAQUE_LEN):
                out += b"\0" * (-len(b) % 4)
        f += 1
    return bytes(out)


def xdr_hashed_stream(schema, msg: bytes):
    """The bytes Mercury's XDR-mode proc checksum covers for one message, or
    None when the schema runs past the message."""
    pos, last, out, f = 0, 0, bytearray(), 0
    while f < len(schema):
        kind, size = schema[f]
        f += 1
        if kind == XDR_SKIP_IF_ZERO:
            if last == 0:
                f += size
            continue
        if kind == XDR_INT:
            slot = 4 if size <= 4 else 8
            if pos + slot > len(msg):
                return None
            v = int.from_bytes(msg[pos:pos + slot], "big")
            out += (v & ((1 << (8 * size)) - 1)).to_bytes(size, "little")
            last = v & ((1 << (8 * size)) - 1)
            pos += slot
            continue
        n = last if kind in (XDR_OPAQUE_LEN, XDR_RAW_LEN) else size
        wire = n if kind in (XDR_RAW, XDR_RAW_LEN) else n + (-n % 4)
        if pos + wire > len(msg):
            return None
        out += msg[pos:pos + n]
        pos += wire
    return bytes(out)
