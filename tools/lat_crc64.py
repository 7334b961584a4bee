#!/usr/bin/env python3
"""Small-batch latency of the CRC-64 batch entry point (fixed 4 KiB payloads):
per-call device time by HIP events.  CRC-64 has no light layout; this shows
what the throughput layout costs per call at small batch sizes."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G


def main():
    length = 4096
    G.prepare("crc64")
    big = torch.empty(16384 * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(big, 1)
    res = []
    for count in (1, 8, 64, 256, 1024, 4096, 16384):
        out = torch.empty(count, dtype=torch.int64, device="cuda")
        f = lambda: G.checksum_fixed("crc64", big, length, count=count, out=out)  # noqa: E731
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
        for a, b in ev:
            a.record(s)
            f()
            b.record(s)
        torch.cuda.synchronize()
        dev_us = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
        res.append({"method": "crc64", "payloads": count, "bytes": count * length, "device_us": round(dev_us, 2),
                    "GBps_device": round(count * length / dev_us / 1e3, 1)})
        print(json.dumps(res[-1]), flush=True)
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
