"""Python view of the streaming mchecksum API (include/mchecksum.h).

Mirrors the upstream C surface one to one -- init / reset / update / get /
get_size / destroy, method names "crc16", "crc32c", "crc64" -- so tests read
like Mercury's own use of it (src/mercury_proc.c:34-99, 151-217, 358-472).
"""
from __future__ import annotations

import ctypes

from ._lib import load_library

MCHECKSUM_FINALIZE = 1


class MChecksumError(RuntimeError):
    pass


class Checksum:
    """One mchecksum object (struct mchecksum_object *)."""

    def __init__(self, hash_method: str):
        self._lib = load_library()
        self._obj = ctypes.c_void_p()
        rc = self._lib.mchecksum_init(hash_method.encode(), ctypes.byref(self._obj))
        if rc != 0:
            raise MChecksumError(f"mchecksum_init({hash_method!r}) failed")
        self.method = hash_method

    def reset(self) -> None:
        if self._lib.mchecksum_reset(self._obj) != 0:
            raise MChecksumError("mchecksum_reset failed")

    def get_size(self) -> int:
        return int(self._lib.mchecksum_get_size(self._obj))

    def update(self, data) -> None:
        b = bytes(data)
        buf = ctypes.create_string_buffer(b, len(b)) if b else None
        if self._lib.mchecksum_update(self._obj, buf, len(b)) != 0:
            raise MChecksumError("mchecksum_update failed")

    def get_bytes(self, size: int | None = None, finalize: int = MCHECKSUM_FINALIZE) -> bytes:
        size = self.get_size() if size is None else size
        buf = ctypes.create_string_buffer(max(size, 1))
        if self._lib.mchecksum_get(self._obj, buf, size, finalize) != 0:
            raise MChecksumError("mchecksum_get failed")
        return buf.raw[:self.get_size()]

    def get(self) -> int:
        """The checksum as the host-order integer mchecksum_get writes."""
        return int.from_bytes(self.get_bytes(), "little")

    def close(self) -> None:
        if self._obj:
            self._lib.mchecksum_destroy(self._obj)
            self._obj = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def checksum(hash_method: str, data) -> int:
    c = Checksum(hash_method)
    try:
        c.update(data)
        return c.get()
    finally:
        c.close()
