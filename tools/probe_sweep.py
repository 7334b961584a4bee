#!/usr/bin/env python3
"""DIAGNOSTIC: HBM read ceiling by access pattern (tools/hbm_probe.hip)."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G
P = ctypes.CDLL(os.path.join(ROOT, "build", "libhbm_probe.so"))
P.hbm_probe2.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_void_p]
count, length = 65536, 65536
data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
G.fill_splitmix(data, 5)
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
out = torch.empty(count, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
cfgs = []
for nt in (1, 0):
    for mode in (0, 1):
        for unr in (4, 8):
            for bpc, thr in ((1, 1024), (2, 1024), (4, 512), (8, 256)):
                cfgs.append((nt, mode, unr, bpc, thr))
res = {c: [] for c in cfgs}
res["crc"] = []
G.prepare("crc32c")
for rnd in range(4):
    for c in cfgs:
        nt, mode, unr, bpc, thr = c
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(6)]
        for a, b in ev:
            a.record(s)
            P.hbm_probe2(data.data_ptr(), length, count, sink.data_ptr(), nt, mode, unr, cus * bpc, thr, s.cuda_stream)
            b.record(s)
        torch.cuda.synchronize()
        if rnd:
            res[c] += [a.elapsed_time(b) for a, b in ev]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(6)]
    for a, b in ev:
        a.record(s); G.checksum_fixed("crc32c", data, length, count=count, out=out); b.record(s)
    torch.cuda.synchronize()
    if rnd:
        res["crc"] += [a.elapsed_time(b) for a, b in ev]
for c, v in sorted(res.items(), key=lambda kv: np.median(kv[1])):
    v = np.array(v)
    name = "crc32c kernel" if c == "crc" else "nt=%d mode=%s unroll=%d blocks/CU=%d threads=%d" % (c[0], "payload" if c[1] == 0 else "linear", c[2], c[3], c[4])
    print(f"{name:58s} median {np.median(v):.4f} ms = {count*length/np.median(v)/1e6:.0f} GB/s  (best {count*length/v.min()/1e6:.0f})")
