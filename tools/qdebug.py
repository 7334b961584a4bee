#!/usr/bin/env python3
"""Small launches through a -DMCK_TRACE=1 build (bounded queue spins): checks
results against the default library's light path and prints any spin-guard
records (kind 1 = ring recycle wait, 2 = chunk publication wait)."""
import ctypes, os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_variants import load  # noqa: E402
from mercury_amd import gpu as G  # noqa: E402

lib = load(os.path.join(ROOT, "build", "variants", "libmchecksum_trace.so"))
lib.mck_debug_qdiag_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
s = torch.cuda.current_stream().cuda_stream
CASES = [("crc32c", 67, 65536), ("crc32c", 16, 65536), ("crc32c", 17, 65536), ("crc32c", 1, 65536), ("crc32c", 67, 4096), ("crc64", 67, 4096), ("crc32c", 4096, 4096)]
for method, count, length in CASES:
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, 7)
    os.environ["MCHECKSUM_GPU_LIGHT"] = "0"
    o = torch.zeros(count, dtype=torch.int32 if method == "crc32c" else torch.int64, device="cuda")
    rc = lib.mchecksum_gpu_checksum_fixed(method.encode(), data.data_ptr(), length, length, count, o.data_ptr(), s)
    ev = torch.cuda.Event()
    ev.record()
    t0 = time.time()
    while not ev.query():
        if time.time() - t0 > 20:
            print("HUNG: kernel not done after 20 s", method, count, length, flush=True)
            os._exit(3)
        time.sleep(0.01)
    torch.cuda.synchronize()
    os.environ["MCHECKSUM_GPU_LIGHT"] = "1" if method == "crc32c" else "0"
    ref = G.checksum_fixed(method, data, length, count=count)
    torch.cuda.synchronize()
    n = ctypes.c_uint(0)
    rec = np.zeros(256, dtype=np.uint64)
    lib.mck_debug_qdiag_read(ctypes.byref(n), rec.ctypes.data)
    bad = int((o != ref).sum())
    print(method, count, length, "rc", rc, "mismatches", bad, "spin-guard records", n.value, flush=True)
    for i in range(min(n.value, 8)):
        print("   kind %d wave %d x %d y %#x" % tuple(int(v) for v in rec[4 * i:4 * i + 4]))
