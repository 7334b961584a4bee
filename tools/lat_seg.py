#!/usr/bin/env python3
"""DIAGNOSTIC: per-call device time of mchecksum_gpu_checksum_segments for the
small lists a bulk handle carries, with the scan fused into the chunk pass
(one launch, MCHECKSUM_GPU_SEG_FUSED=1, round 5) and with the separate scan
launch (MCHECKSUM_GPU_SEG_FUSED=0, the default), interleaved in one process.  Per call: one HIP
event pair around 200 back-to-back calls on one prepared SegmentBatch."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402

SHAPES = [(1, 4096), (4, 65536), (16, 262144), (64, 4096), (256, 4096), (1024, 4096), (4, 1 << 20)]


def main():
    data = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, 0x1A7)
    res = {}
    for method in ("crc64", "crc32c"):
        for nseg, ln in SHAPES:
            views = [data[i * ln:(i + 1) * ln] for i in range(nseg)]
            b = G.SegmentBatch(views, [0, nseg])
            out = torch.empty(1, dtype=G.out_dtype(method), device="cuda")
            t = {}
            for rnd in range(3):
                for mode in ("fused", "launch"):
                    os.environ["MCHECKSUM_GPU_SEG_FUSED"] = "1" if mode == "fused" else "0"
                    for _ in range(20):
                        b.checksum(method, out=out)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(200):
                        b.checksum(method, out=out)
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1e3 / 200
                    t[mode] = min(t.get(mode, 1e9), us)
            key = f"{method} {nseg} x {ln} B"
            res[key] = {k: round(v, 2) for k, v in t.items()}
            print(f"{key:28s} fused {t['fused']:8.2f} us   scan launch {t['launch']:8.2f} us")
    os.environ.pop("MCHECKSUM_GPU_SEG_FUSED", None)
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
