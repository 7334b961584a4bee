#!/usr/bin/env python3
"""DIAGNOSTIC: per-launch time of the headline kernel shape (64 KiB CRC-32C
payloads on the work queue) against batch size, 1 to 64 GiB, in interleaved
blocks of one process.  A straight-line fit t = a + bytes / rate separates a
fixed per-launch cost from the streaming rate."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402


def main():
    length = 65536
    sizes = [1, 2, 4, 8, 16, 32, 64]  # GiB
    data = torch.empty((64 << 30) + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, 5)
    G.prepare("crc32c")
    out = torch.empty((64 << 30) // length, dtype=torch.int32, device="cuda")

    def run(gib, n):
        count = (gib << 30) // length
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for i in range(n):
            ev[i][0].record()
            G.checksum_fixed("crc32c", data, length, count=count, out=out)
            ev[i][1].record()
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3  # us

    for _ in range(40):
        run(4, 1)
    res = {g: [] for g in sizes}
    for rnd in range(3):
        for g in (sizes if rnd % 2 == 0 else sizes[::-1]):
            res[g].append(run(g, max(4, 64 // g * 3)))
    t = np.array([np.median(res[g]) for g in sizes])
    b = np.array([g << 30 for g in sizes], dtype=np.float64)
    slope, icpt = np.polyfit(b, t, 1)
    out_d = {"us_per_launch": {str(g): round(float(v), 2) for g, v in zip(sizes, t)},
             "TBps": {str(g): round(float(bb / (v * 1e-6) / 1e12), 3) for g, bb, v in zip(sizes, b, t)},
             "fit_fixed_us": round(float(icpt), 2), "fit_rate_TBps": round(float(1 / slope / 1e6), 3)}
    print(json.dumps(out_d), flush=True)
    json.dump(out_d, open(os.path.join(ROOT, "gpurun_out", "size_sweep.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
