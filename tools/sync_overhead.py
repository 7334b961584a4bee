#!/usr/bin/env python3
"""DIAGNOSTIC: where bench.py's wall-minus-event time goes (headline shape).

bench.py reports value = bytes / wall, with wall = barrier + synchronize on
both sides of the K launches, and kernel_ms from one HIP event pair around
them.  The difference (~160 us per timed region, i.e. 8 us per step at the
driver's K = 20) is host<->device latency at the region's two ends.  This
probe times, interleaved, for K = 20 launches after a 40-launch warm-up:
  sync   : exactly bench.py's bracket (torch.cuda.synchronize() both sides)
  spin   : the same, but the host polls the end event (busy wait) before the
           closing synchronize
and reports wall - events for each.  With SPIN_FLAGS=1 the process first sets
hipDeviceScheduleSpin (hipSetDeviceFlags, before torch creates its context),
so every blocking wait busy-polls.
usage: python tools/sync_overhead.py  (writes gpurun_out/sync_overhead*.json)"""
import ctypes
import json
import os
import sys
import time

if os.environ.get("SPIN_FLAGS") == "1":
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
    print(f"hipSetDeviceFlags(spin) rc={rc}", flush=True)

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402


def main():
    count, length, K = 65536, 65536, 20
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, 0x4D43310000000005)
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(40):
        G.checksum_fixed("crc32c", data, length, count=count, out=out)
    torch.cuda.synchronize()
    res = {"sync": [], "spin": []}
    for rnd in range(12):
        for mode in ("sync", "spin"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(s)
            for _ in range(K):
                G.checksum_fixed("crc32c", data, length, count=count, out=out)
            e1.record(s)
            t_issued = time.perf_counter()
            if mode == "spin":
                while not e1.query():
                    pass
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            ev = e0.elapsed_time(e1)
            res[mode].append({"wall_ms": round(wall, 4), "event_ms": round(ev, 4),
                              "overhead_us": round((wall - ev) * 1e3, 1),
                              "issue_us": round((t_issued - t0) * 1e6, 1)})
    summ = {m: {"median_overhead_us": float(np.median([r["overhead_us"] for r in v])),
                "median_event_ms_per_step": float(np.median([r["event_ms"] for r in v])) / K,
                "median_issue_us": float(np.median([r["issue_us"] for r in v]))} for m, v in res.items()}
    tag = "_spinflags" if os.environ.get("SPIN_FLAGS") == "1" else ""
    doc = {"K": K, "summary": summ, "runs": res, "spin_flags": tag != ""}
    print(json.dumps(summ), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(doc, open(os.path.join(ROOT, "gpurun_out", f"sync_overhead{tag}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
