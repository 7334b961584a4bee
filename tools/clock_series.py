#!/usr/bin/env python3
"""DIAGNOSTIC: shader clock (SCLK) against per-launch time over a series of
back-to-back headline launches (64K x 64 KiB CRC-32C) -- is the slowdown over
the first ~30 launches (profiles/r01/launch_series_metric.json) a clock drop?

A one-wave sampler kernel (tools/clock_probe.hip) runs on a second stream for
the whole series and records (shader-clock counter, 100 MHz real-time counter)
pairs every 2 us; SCLK over an interval = d(shader) / d(real) * 100 MHz.  Each
launch's window comes from HIP events; the sampler's start is aligned to the
series by an event recorded on its stream just before it.

usage: clock_series.py OUT.json [launches] [scenario ...]
scenarios: fresh (right after the data fill, as bench.py), idle (1 s idle
first), probe (the read-only HBM probe kernel instead of the CRC kernel)
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402

OUT = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 60
SCEN = sys.argv[3:] or ["fresh", "idle", "probe"]

P = ctypes.CDLL(os.path.join(ROOT, "build", "libclock_probe.so"))
P.mck_clock_sampler.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_ulonglong,
                                ctypes.c_void_p]
H = None
if "probe" in SCEN:
    H = ctypes.CDLL(os.path.join(ROOT, "build", "libhbm_probe.so"))
    H.hbm_probe.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                            ctypes.c_int, ctypes.c_void_p]

count, length = 65536, 65536
data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
out = torch.empty(count, dtype=torch.int32, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
G.prepare("crc32c")
cus = torch.cuda.get_device_properties(0).multi_processor_count
sa = torch.cuda.current_stream()
sb = torch.cuda.Stream()
NS = 60000
samp = torch.zeros(2 * NS, dtype=torch.int64, device="cuda")


def series(kind):
    samp.zero_()
    torch.cuda.synchronize()
    eb, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(N)]
    eb.record(sb)
    limit = int((N * 0.9 + 5) * 1e5)  # ticks of 10 ns: ~0.9 ms per launch + 5 ms
    assert P.mck_clock_sampler(samp.data_ptr(), NS, 200, limit, sb.cuda_stream) == 0
    e0.record(sa)
    for a, b in ev:
        a.record(sa)
        if kind == "probe":
            H.hbm_probe(data.data_ptr(), length, count, sink.data_ptr(), 1, cus, sa.cuda_stream)
        else:
            G.checksum_fixed("crc32c", data, length, count=count, out=out)
        b.record(sa)
    torch.cuda.synchronize()
    s = samp.cpu().numpy().astype(np.uint64).reshape(-1, 2)
    s = s[s[:, 1] != 0]
    clk = np.diff(s[:, 0].astype(np.float64))
    rt = np.diff(s[:, 1].astype(np.float64))
    mhz = clk / rt * 100.0
    t_ms = (s[1:, 1].astype(np.float64) - float(s[0, 1])) * 1e-5  # end of each interval, ms from sampler start
    off = eb.elapsed_time(e0)  # sampler start -> series start (ms)
    starts = np.array([e0.elapsed_time(a) for a, _ in ev]) + off
    ends = np.array([e0.elapsed_time(b) for _, b in ev]) + off
    per = []
    for lo, hi in zip(starts, ends):
        m = (t_ms > lo) & (t_ms <= hi)
        per.append(float(np.mean(mhz[m])) if m.any() else None)
    dur = (ends - starts).tolist()
    bins = {}
    for lo in np.arange(0, float(ends[-1]) + 0.5, 0.5):
        m = (t_ms > lo) & (t_ms <= lo + 0.5)
        if m.any():
            bins[f"{lo:.1f}"] = round(float(np.mean(mhz[m])), 1)
    idle = t_ms <= starts[0]
    return {"launch_ms": [round(x, 4) for x in dur], "launch_sclk_mhz": [round(x, 1) if x else None for x in per],
            "sclk_before_series_mhz": round(float(np.mean(mhz[idle])), 1) if idle.any() else None,
            "sclk_timeline_0p5ms": bins, "samples": int(len(s))}


res = {"launches": N, "device": torch.cuda.get_device_name(0)}
for sc in SCEN:
    G.fill_splitmix(data, 0x4D43310000000005)
    if sc == "idle":
        torch.cuda.synchronize()
        time.sleep(1.0)
    r = series("probe" if sc == "probe" else "crc")
    res[sc] = r
    d, f = np.array(r["launch_ms"]), r["launch_sclk_mhz"]
    print(f"{sc}: launches 0-4 {d[:5].mean():.3f} ms, 5-15 {d[5:15].mean():.3f}, 15-30 {d[15:30].mean():.3f}, "
          f"30+ {d[30:].mean():.3f}; SCLK idle {r['sclk_before_series_mhz']} MHz, per launch "
          + " ".join(f"{x:.0f}" if x else "-" for x in f[:40]), flush=True)
json.dump(res, open(OUT, "w"), indent=1)
