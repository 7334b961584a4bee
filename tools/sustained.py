#!/usr/bin/env python3
"""DIAGNOSTIC: sustained per-launch times of the CRC-32C batch kernel vs the
read-only HBM probe (tools/hbm_probe.hip) on the headline 64K x 64 KiB batch,
in alternating blocks within one process."""
import ctypes, json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G

P = ctypes.CDLL(os.path.join(ROOT, "build", "libhbm_probe.so"))
P.hbm_probe.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                        ctypes.c_int, ctypes.c_void_p]
count, length = 65536, 65536
data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
G.fill_splitmix(data, 0x4D43310000000005)
out = torch.empty(count, dtype=torch.int32, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
blocks = torch.cuda.get_device_properties(0).multi_processor_count
G.prepare("crc32c")
runs = {
    "crc_nt": lambda: G.checksum_fixed("crc32c", data, length, count=count, out=out),
    "probe_nt": lambda: P.hbm_probe(data.data_ptr(), length, count, sink.data_ptr(), 1, blocks, s.cuda_stream),
    "probe_plain": lambda: P.hbm_probe(data.data_ptr(), length, count, sink.data_ptr(), 0, blocks, s.cuda_stream),
}
def crc_plain():
    os.environ["MCHECKSUM_GPU_NT"] = "0"
    G.checksum_fixed("crc32c", data, length, count=count, out=out)
    del os.environ["MCHECKSUM_GPU_NT"]
runs["crc_plain"] = crc_plain
n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
res = {k: [] for k in runs}
for rnd in range(3):
    for k, f in runs.items():
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for a, b in ev:
            a.record(s); f(); b.record(s)
        torch.cuda.synchronize()
        res[k] += [a.elapsed_time(b) for a, b in ev]
for k, v in res.items():
    v = np.array(v)
    print(f"{k:12s} median {np.median(v):.4f} ms p10 {np.percentile(v,10):.4f} p90 {np.percentile(v,90):.4f} "
          f"-> median {count*length/np.median(v)/1e6:.0f} GB/s, p10 {count*length/np.percentile(v,10)/1e6:.0f} GB/s")
    print("   first 12:", " ".join(f"{x:.3f}" for x in v[:12]))
json.dump({k: list(map(float, v)) for k, v in res.items()}, open(os.path.join(ROOT, "gpurun_out", "sustained.json"), "w"))
