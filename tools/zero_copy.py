#!/usr/bin/env python3
"""Checksum rate of byte-packed payloads that live in HOST memory (Mercury's
NA receive buffers and proc buffers: SURVEY.md 8(f)1, north_star's "starts
and ends in host memory"), three ways, on a C4-mix sample:

  zero_copy  -- the buffer registered once (hipHostRegister, Mapped) and its
                device alias passed straight to mchecksum_gpu_checksum_offsets:
                the kernel reads the bytes over PCIe, no staging copy;
  staged     -- one hipMemcpyAsync of the whole sample to device memory, then
                the device-resident kernel (the copy dominates);
  device     -- the kernel on the device-resident copy (the HBM roofline leg);
and the oracle's SSE4.2 crc32c on the host's cores for the same bytes.
Every path's CRCs are checked against the oracle.  Output: one JSON object.

usage: zero_copy.py [--mib 1024] [--iters 10] [--out FILE]
"""
import argparse
import ctypes
import json
import mmap
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402
from mercury_amd.workload import varlen_offsets  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    seed = 0x4D43310000000004
    full = varlen_offsets(seed, 262144)
    n = int(np.searchsorted(full, np.uint64(args.mib << 20)))
    off = np.ascontiguousarray(full[:n + 1])
    nbytes = int(off[-1])
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    vp = ctypes.c_void_p
    hip.hipHostRegister.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [vp]
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_uint]
    hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]

    mm = mmap.mmap(-1, nbytes + 64)
    host = np.frombuffer(mm, dtype=np.uint8)
    host[:nbytes] = O.splitmix_bytes(nbytes, seed)
    hptr = ctypes.addressof(ctypes.c_char.from_buffer(mm))
    t0 = time.perf_counter()
    assert hip.hipHostRegister(hptr, nbytes + 64, 0x2) == 0  # once per buffer, as an NA plugin would
    reg_ms = (time.perf_counter() - t0) * 1e3
    d = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(d), hptr, 0) == 0
    alias = d.value

    lib = G._lib()
    offs = torch.from_numpy(off.astype(np.int64)).cuda()
    dev = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    G.prepare("crc32c")
    want = O.batch_offsets("crc32c", host[:nbytes], off, variant="sse42", nthreads=16)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(args.iters):
            fn()
        b.record(s)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / args.iters

    def zero_copy():
        assert lib.mchecksum_gpu_checksum_offsets(b"crc32c", alias, offs.data_ptr(), n, out.data_ptr(), sh) == 0

    def staged():
        assert hip.hipMemcpyAsync(dev.data_ptr(), hptr, nbytes, 1, sh) == 0  # hipMemcpyHostToDevice
        assert lib.mchecksum_gpu_checksum_offsets(b"crc32c", dev.data_ptr(), offs.data_ptr(), n, out.data_ptr(), sh) == 0

    def device():
        assert lib.mchecksum_gpu_checksum_offsets(b"crc32c", dev.data_ptr(), offs.data_ptr(), n, out.data_ptr(), sh) == 0

    res = {"payloads": n, "bytes": nbytes, "register_ms": round(reg_ms, 1)}
    for name, fn in (("zero_copy", zero_copy), ("staged", staged), ("device", device)):
        ms = timed(fn)
        ok = np.array_equal(G.as_unsigned(out).astype(np.uint64), want)
        res[name] = {"ms": round(ms, 4), "GB_s": round(nbytes / ms / 1e6, 1), "oracle_exact": bool(ok)}
        print(name, res[name], flush=True)
    laps = []
    for _ in range(5):
        t = time.perf_counter()
        O.batch_offsets("crc32c", host[:nbytes], off, variant="sse42", nthreads=16)
        laps.append(time.perf_counter() - t)
    res["cpu_sse42_16_threads"] = {"ms": round(float(np.median(laps)) * 1e3, 2),
                                   "GB_s": round(nbytes / float(np.median(laps)) / 1e9, 1)}
    print("cpu", res["cpu_sse42_16_threads"], flush=True)
    assert hip.hipHostUnregister(hptr) == 0
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
