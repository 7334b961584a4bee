#!/usr/bin/env python3
"""DIAGNOSTIC: small-batch calls for a rocprofv3 kernel trace (device time per
kernel vs event-measured time)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G
G.prepare("crc32c")
big = torch.empty(4096 * 4096 + 64, dtype=torch.uint8, device="cuda")
G.fill_splitmix(big, 1)
for count in (1, 1024):
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    for _ in range(50):
        G.checksum_fixed("crc32c", big, 4096, count=count, out=out)
    torch.cuda.synchronize()
x = torch.zeros(16, device="cuda")
for _ in range(50):
    x.add_(1)
torch.cuda.synchronize()
print("ok")
