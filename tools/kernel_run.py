#!/usr/bin/env python3
"""DIAGNOSTIC: run one config's batch kernel N times (for rocprofv3 --pmc passes)."""
import argparse, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from mercury_amd import gpu as G
from tools_shapes import SHAPES
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
method, count, length, seed = SHAPES[a.config]
if length is None:
    from mercury_amd.workload import varlen_offsets
    off = varlen_offsets(seed, count)
    data = torch.empty(int(off[-1]) + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    offs = torch.from_numpy(off.astype(np.int64)).cuda()
    run = lambda: G.checksum_offsets(method, data, offs)
else:
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    run = lambda: G.checksum_fixed(method, data, length, count=count)
for _ in range(a.iters):
    run()
torch.cuda.synchronize()
print("ok")
