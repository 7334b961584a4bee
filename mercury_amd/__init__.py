"""mercury_amd -- MI355X-native mchecksum for Mercury's RPC checksum path.

libmchecksum.so exports the unchanged mchecksum C ABI Mercury links when built
with MERCURY_USE_CHECKSUMS=ON (include/mchecksum.h) plus MI355X batch entry
points for device-resident payloads (include/mchecksum_gpu.h).  This package
is the Python view of that library: `mchecksum` mirrors the streaming API,
`gpu` drives the batch kernels on torch device memory.
"""
from ._lib import LIB_PATH, load_library  # noqa: F401
from .mchecksum import Checksum, checksum  # noqa: F401

__all__ = ["LIB_PATH", "load_library", "Checksum", "checksum"]
