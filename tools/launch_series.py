#!/usr/bin/env python3
"""DIAGNOSTIC: per-launch device time of N back-to-back headline launches
(64K x 64 KiB CRC-32C) -- the DVFS shape bench.py's mean averages over."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
count, length = 65536, 65536
data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
G.fill_splitmix(data, 0x4D43310000000005)
out = torch.empty(count, dtype=torch.int32, device="cuda")
G.prepare("crc32c")
torch.cuda.synchronize()
s = torch.cuda.current_stream()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
for a, b in ev:
    a.record(s)
    G.checksum_fixed("crc32c", data, length, count=count, out=out)
    b.record(s)
torch.cuda.synchronize()
t = np.array([a.elapsed_time(b) for a, b in ev])
print("per-launch ms:", " ".join(f"{x:.3f}" for x in t))
for lo, hi in ((0, 10), (10, 60), (30, 80), (60, n)):
    print(f"launches [{lo},{min(hi, n)}): mean {t[lo:hi].mean():.4f} ms, median {np.median(t[lo:hi]):.4f} ms")
json.dump(t.tolist(), open(os.path.join(ROOT, "gpurun_out", "launch_series.json"), "w"))
