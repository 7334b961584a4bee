#!/usr/bin/env python3
"""DIAGNOSTIC: which scatter-gather object shapes disagree with the oracle."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G
from oracle import oracle as O
buf = torch.empty((4 << 20) + 64, dtype=torch.uint8, device="cuda")
G.fill_splitmix(buf, 99)
host = buf.cpu().numpy()
for method in ("crc32c", "crc64"):
    for shape in ([1], [5], [100], [4096], [300000], [0], [1, 1], [8, 8], [100, 7], [4096, 4096], [300000, 5], [5, 300000]):
        segs, off = [], 17
        for n in shape:
            segs.append((off, n)); off += n + 33
        got = int(G.as_unsigned(G.checksum_segments(method, [buf[o:o + n] for o, n in segs]))[0])
        want = O.crc(method, np.concatenate([host[o:o + n] for o, n in segs]) if segs else np.zeros(0, np.uint8))
        print(method, shape, "ok" if got == want else f"BAD got {got:x} want {want:x}")
