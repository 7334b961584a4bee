#!/usr/bin/env python3
"""DIAGNOSTIC: does the headline launch (65536 x 64 KiB CRC-32C) stream
faster when consecutive launches read different 4 GiB windows of a 64 GiB
buffer instead of the same 4 GiB?  (The 64 GiB C5 launch streams ~3% faster
than the 4 GiB headline.)  Alternates blocks of 50 launches: same window /
rotating windows / one 64 GiB launch, after 40 warm-up launches."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402


def main():
    count, length, win = 65536, 65536, 16
    data = torch.empty(win * count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, 5)
    G.prepare("crc32c")
    out = torch.empty(win * count, dtype=torch.int32, device="cuda")
    wb = count * length

    def launch(w):
        G.checksum_fixed("crc32c", data[w * wb:(w + 1) * wb + 64], length, count=count, out=out[w * count:(w + 1) * count])

    def timed(kind, n=50):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for i in range(n):
            ev[i][0].record()
            if kind == "same":
                launch(0)
            elif kind == "rotate":
                launch(i % win)
            else:
                G.checksum_fixed("crc32c", data, length, count=win * count, out=out)
            ev[i][1].record()
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in ev]
        nbytes = (win if kind == "c5" else 1) * wb
        return round(float(np.mean(ms)), 4), round(nbytes / (np.mean(ms) * 1e-3) / 1e12, 3)

    for i in range(40):
        launch(i % win)
    torch.cuda.synchronize()
    res = {"same": [], "rotate": [], "c5": []}
    for rnd in range(4):
        for kind in ("same", "rotate") if rnd % 2 == 0 else ("rotate", "same"):
            res[kind].append(timed(kind))
        res["c5"].append(timed("c5", 6))
    for k, v in res.items():
        print(k, "mean_ms/TBps per block:", v, flush=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "footprint_probe.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
