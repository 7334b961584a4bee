#!/usr/bin/env python3
"""DIAGNOSTIC A/B for the start of a launch series (the driver's bench run:
5 warm-up + 20 timed launches of the 64K x 64 KiB headline, right after the
data fill).  Over those launches the shader clock falls from 2.4 GHz to
~1.0 GHz and climbs back (tools/clock_series.py), so what a variant does per
CLOCK there -- not its steady-state HBM-bound time -- sets the number.

Per round and variant (interleaved, rounds rotate the order): 1 s idle, then
W + K launches with HIP events and the SCLK sampler (tools/clock_probe.hip)
running beside them, then 40 more launches (steady state).  Reports per
variant: median over rounds of the timed-launch mean, the mean SCLK over the
timed launches, bytes per shader clock per CU, and the steady-state mean.
Every variant's CRCs must equal the first one's.

usage: hump_ab.py OUT.json variant ... (names of build/variants/libmchecksum_<name>.so)
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

OUT, NAMES = sys.argv[1], sys.argv[2:]
W, K, ROUNDS, STEADY = 5, 20, int(os.environ.get("ROUNDS", "4")), 40
CFG = os.environ.get("CFG", "metric")
SHAPE = {"metric": ("crc32c", 65536, 65536, 0x4D43310000000005), "c2": ("crc32c", 65536, 4096, 0x4D43310000000002),
         "c3": ("crc64", 8192, 1 << 20, 0x4D43310000000003)}[CFG]
method, count, length, seed = SHAPE

P = ctypes.CDLL(os.path.join(ROOT, "build", "libclock_probe.so"))
P.mck_clock_sampler.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_ulonglong,
                                ctypes.c_void_p]
libs = []
for n in NAMES:
    L = ctypes.CDLL(os.path.join(ROOT, "build", "variants", f"libmchecksum_{n}.so"))
    L.mchecksum_gpu_prepare.argtypes = [ctypes.c_char_p]
    L.mchecksum_gpu_checksum_fixed.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                               ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    assert L.mchecksum_gpu_prepare(method.encode()) == 0
    libs.append(L)

data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
G.fill_splitmix(data, seed)
outs = [torch.empty(count, dtype=G.out_dtype(method), device="cuda") for _ in libs]
cus = torch.cuda.get_device_properties(0).multi_processor_count
sa = torch.cuda.current_stream()
sb = torch.cuda.Stream()
NS = 40000
samp = torch.zeros(2 * NS, dtype=torch.int64, device="cuda")
nbytes = count * length


def run_series(L, out):
    samp.zero_()
    torch.cuda.synchronize()
    time.sleep(1.0)
    eb, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = W + K + STEADY
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    eb.record(sb)
    assert P.mck_clock_sampler(samp.data_ptr(), NS, 200, int((W + K) * 2e5 + 5e5), sb.cuda_stream) == 0
    e0.record(sa)
    for a, b in ev:
        a.record(sa)
        assert L.mchecksum_gpu_checksum_fixed(method.encode(), data.data_ptr(), length, length, count,
                                              out.data_ptr(), sa.cuda_stream) == 0
        b.record(sa)
    torch.cuda.synchronize()
    s = samp.cpu().numpy().astype(np.uint64).reshape(-1, 2)
    s = s[s[:, 1] != 0]
    mhz = np.diff(s[:, 0].astype(np.float64)) / np.diff(s[:, 1].astype(np.float64)) * 100.0
    t_ms = (s[1:, 1].astype(np.float64) - float(s[0, 1])) * 1e-5
    off = eb.elapsed_time(e0)
    st = np.array([e0.elapsed_time(a) for a, _ in ev]) + off
    en = np.array([e0.elapsed_time(b) for _, b in ev]) + off
    dur = en - st
    m = (t_ms > st[W]) & (t_ms <= en[W + K - 1])
    f = float(np.mean(mhz[m])) if m.any() else float("nan")
    timed = float(dur[W:W + K].mean())
    return {"timed_ms": timed, "sclk_mhz": f, "steady_ms": float(dur[-20:].mean()),
            "b_per_clk_cu": nbytes / (timed * 1e-3) / (f * 1e6) / cus, "dur": dur.round(4).tolist()}


res = {n: [] for n in NAMES}
for r in range(ROUNDS):
    order = list(range(len(libs)))
    order = order[r % len(order):] + order[:r % len(order)]
    for i in order:
        res[NAMES[i]].append(run_series(libs[i], outs[i]))
ref = G.as_unsigned(outs[0])
summary = {}
for i, n in enumerate(NAMES):
    same = bool(np.array_equal(G.as_unsigned(outs[i]), ref))
    rs = res[n]
    summary[n] = {k: round(float(np.median([x[k] for x in rs])), 4) for k in ("timed_ms", "sclk_mhz", "steady_ms",
                                                                            "b_per_clk_cu")}
    summary[n]["crc_equal"] = same
    summary[n]["GiB_s_timed"] = round(nbytes / (summary[n]["timed_ms"] * 1e-3) / 2**30, 1)
    print(n, json.dumps(summary[n]), flush=True)
json.dump({"config": CFG, "W": W, "K": K, "rounds": ROUNDS, "summary": summary, "raw": res}, open(OUT, "w"))
