#!/usr/bin/env python3
"""Host cost of issuing one batch call, against the device time of the call.

A step of bench.py is one Python call of mercury_amd.gpu (argument checks, the
device guard, ctypes, the C entry point, hipLaunchKernel).  When that costs
more than the kernel runs, the GPU idles between launches and both the wall
time and the event-bracketed kernel time include the gap.  This enqueues N
calls without synchronising and reports host microseconds per call for:
  wrapper  -- mercury_amd.gpu.checksum_fixed (what bench.py calls)
  ctypes   -- the C entry point called directly through ctypes
  torch    -- a trivial torch kernel (out.zero_()) for scale
and the device time per call from one event pair around N back-to-back calls.

usage: host_overhead.py [--config c2|metric] [--n 400] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402
from mercury_amd._lib import load_library  # noqa: E402

SHAPES = {"c2": (65536, 4096, 0x4D43310000000002), "metric": (65536, 65536, 0x4D43310000000005)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    count, length, seed = SHAPES[a.config]
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    G.checksum_fixed("crc32c", data, length, count=count, out=out)
    ref = out.clone()
    L = load_library()
    s = torch.cuda.current_stream()
    h = s.cuda_stream
    m = b"crc32c"
    dp, op = data.data_ptr(), out.data_ptr()

    calls = {
        "wrapper": lambda: G.checksum_fixed("crc32c", data, length, count=count, out=out),
        "ctypes": lambda: L.mchecksum_gpu_checksum_fixed(m, dp, length, length, count, op, h),
        "torch_zero": lambda: out.zero_(),
    }
    res = {}
    for rnd in range(3):
        for name, f in calls.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            t0 = time.perf_counter()
            for _ in range(a.n):
                f()
            t1 = time.perf_counter()
            e1.record(s)
            torch.cuda.synchronize()
            if rnd:
                r = res.setdefault(name, {"host_us": [], "device_us": []})
                r["host_us"].append((t1 - t0) / a.n * 1e6)
                r["device_us"].append(e0.elapsed_time(e1) / a.n * 1e3)
    G.checksum_fixed("crc32c", data, length, count=count, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    summary = {k: {"host_us_per_call": round(min(v["host_us"]), 2), "device_us_per_call": round(min(v["device_us"]), 2)}
               for k, v in res.items()}
    summary["config"] = a.config
    summary["n"] = a.n
    print(json.dumps(summary, indent=1))
    if a.out:
        json.dump(summary, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
