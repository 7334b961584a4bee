"""Loads libmchecksum.so -- the drop-in mchecksum C ABI plus the MI355X batch
entry points (include/mchecksum.h, include/mchecksum_gpu.h).

There is no Python or CPU fallback for the batch path: if the shared library
is missing the import fails loudly; if no HIP device is usable, every batch
call raises (MCHECKSUM_GPU_ENODEV).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libmchecksum.so")
BENCH_LIB_PATH = os.path.join(LIB_DIR, "libmchecksum_bench.so")

# Every function the public headers declare (checked against include/*.h by
# tests/test_capi.py).
STREAMING_SYMBOLS = ("mchecksum_init", "mchecksum_destroy", "mchecksum_reset", "mchecksum_get_size",
                     "mchecksum_get", "mchecksum_update")
GPU_SYMBOLS = ("mchecksum_gpu_available", "mchecksum_gpu_prepare", "mchecksum_gpu_checksum_fixed",
               "mchecksum_gpu_checksum_offsets", "mchecksum_gpu_verify_offsets", "mchecksum_gpu_verify_messages",
               "mchecksum_gpu_lanes_per_payload", "mchecksum_gpu_last_error", "mchecksum_gpu_segments_work_size",
               "mchecksum_gpu_checksum_segments", "mchecksum_gpu_verify_core_headers",
               "mchecksum_gpu_queue_faults", "mchecksum_gpu_set_error_word", "mchecksum_gpu_checksum_xdr",
               "mchecksum_gpu_queue_stats", "mchecksum_gpu_reload_settings")
CORE_HEADER_REQUEST, CORE_HEADER_RESPONSE = 0, 1
# XDR schema field kinds (include/mchecksum_gpu.h)
XDR_INT, XDR_OPAQUE, XDR_OPAQUE_LEN, XDR_RAW, XDR_RAW_LEN, XDR_SKIP_IF_ZERO = 0, 1, 2, 3, 4, 5


class XdrField(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("size", ctypes.c_uint32)]

_lib = None
_bench = None

c_void_p, c_size_t, c_int, c_char_p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_char_p


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: build it with `make` (or __graft_entry__.build()); "
                          "mercury_amd has no fallback implementation")
    L = ctypes.CDLL(path)
    L.mchecksum_init.argtypes = [c_char_p, ctypes.POINTER(c_void_p)]
    L.mchecksum_init.restype = c_int
    L.mchecksum_destroy.argtypes = [c_void_p]
    L.mchecksum_destroy.restype = c_int
    L.mchecksum_reset.argtypes = [c_void_p]
    L.mchecksum_reset.restype = c_int
    L.mchecksum_get_size.argtypes = [c_void_p]
    L.mchecksum_get_size.restype = c_size_t
    L.mchecksum_get.argtypes = [c_void_p, c_void_p, c_size_t, c_int]
    L.mchecksum_get.restype = c_int
    L.mchecksum_update.argtypes = [c_void_p, c_void_p, c_size_t]
    L.mchecksum_update.restype = c_int
    L.mchecksum_gpu_available.argtypes = []
    L.mchecksum_gpu_available.restype = c_int
    L.mchecksum_gpu_prepare.argtypes = [c_char_p]
    L.mchecksum_gpu_prepare.restype = c_int
    L.mchecksum_gpu_checksum_fixed.argtypes = [c_char_p, c_void_p, c_size_t, c_size_t, c_size_t, c_void_p, c_void_p]
    L.mchecksum_gpu_checksum_fixed.restype = c_int
    L.mchecksum_gpu_checksum_offsets.argtypes = [c_char_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]
    L.mchecksum_gpu_checksum_offsets.restype = c_int
    L.mchecksum_gpu_verify_offsets.argtypes = [c_char_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                               c_void_p, c_void_p]
    L.mchecksum_gpu_verify_offsets.restype = c_int
    L.mchecksum_gpu_verify_messages.argtypes = [c_char_p, c_void_p, c_void_p, c_size_t, c_size_t, c_size_t, c_void_p,
                                                c_void_p, c_void_p]
    L.mchecksum_gpu_verify_messages.restype = c_int
    L.mchecksum_gpu_lanes_per_payload.argtypes = [c_char_p, c_size_t]
    L.mchecksum_gpu_lanes_per_payload.restype = c_int
    L.mchecksum_gpu_segments_work_size.argtypes = [c_size_t]
    L.mchecksum_gpu_segments_work_size.restype = c_size_t
    L.mchecksum_gpu_checksum_segments.argtypes = [c_char_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t,
                                                  c_void_p, c_size_t, c_void_p, c_void_p]
    L.mchecksum_gpu_checksum_segments.restype = c_int
    L.mchecksum_gpu_verify_core_headers.argtypes = [c_char_p, c_int, c_void_p, c_void_p, c_size_t, c_void_p,
                                                    c_void_p, c_void_p]
    L.mchecksum_gpu_verify_core_headers.restype = c_int
    L.mchecksum_gpu_last_error.argtypes = []
    L.mchecksum_gpu_last_error.restype = c_char_p
    L.mchecksum_gpu_queue_faults.argtypes = []
    L.mchecksum_gpu_queue_faults.restype = ctypes.c_longlong
    L.mchecksum_gpu_queue_stats.argtypes = [c_void_p, c_size_t]
    L.mchecksum_gpu_queue_stats.restype = c_int
    L.mchecksum_gpu_set_error_word.argtypes = [c_void_p]
    L.mchecksum_gpu_set_error_word.restype = c_int
    L.mchecksum_gpu_checksum_xdr.argtypes = [c_char_p, ctypes.POINTER(XdrField), c_size_t, c_void_p, c_void_p,
                                             c_size_t, c_void_p, c_void_p, c_void_p]
    L.mchecksum_gpu_checksum_xdr.restype = c_int
    L.mchecksum_gpu_reload_settings.argtypes = []
    L.mchecksum_gpu_reload_settings.restype = None
    _lib = L
    return L


def reload_settings() -> None:
    """Have libmchecksum re-read its MCHECKSUM_* environment settings, which it
    otherwise reads once per process (tests and A/B tools that change them)."""
    load_library().mchecksum_gpu_reload_settings()


# The sources libmchecksum is built from (the Makefile's STAMP_SRCS): their
# digest is compiled into each library (tools/src_digest.py), so a loaded
# library can be checked against the tree beside it.
_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def tree_source_digest() -> str:
    """sha256 over (path, NUL, bytes, NUL) of mercury_amd/csrc/*.{c,h,hip} and
    include/*.h in path order -- tools/src_digest.py's algorithm."""
    import glob
    import hashlib
    paths = []
    for pat in ("mercury_amd/csrc/*.c", "mercury_amd/csrc/*.h", "mercury_amd/csrc/*.hip", "include/*.h"):
        paths += glob.glob(os.path.join(_ROOT, pat))
    h = hashlib.sha256()
    for rel in sorted(os.path.relpath(p, _ROOT) for p in paths):
        h.update(rel.encode() + b"\0")
        with open(os.path.join(_ROOT, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


def library_source_digest(lib: ctypes.CDLL) -> str:
    """The source digest compiled into a loaded libmchecksum build."""
    return (ctypes.c_char * 65).in_dll(lib, "mchecksum_build_source_digest").value.decode()


def load_bench_library(path: str = BENCH_LIB_PATH) -> ctypes.CDLL:
    global _bench
    if _bench is not None:
        return _bench
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: build it with `make`")
    B = ctypes.CDLL(path)
    B.mck_bench_fill_splitmix.argtypes = [c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, c_void_p]
    B.mck_bench_fill_splitmix.restype = c_int
    B.mck_bench_host_alloc.argtypes = [ctypes.c_uint64]
    B.mck_bench_host_alloc.restype = c_void_p
    B.mck_bench_host_free.argtypes = [c_void_p]
    B.mck_bench_host_free.restype = c_int
    B.mck_bench_gate.argtypes = [c_void_p, c_void_p, ctypes.c_double, c_void_p]
    B.mck_bench_gate.restype = c_int
    _bench = B
    return B
