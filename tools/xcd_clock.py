#!/usr/bin/env python3
"""Per-XCD end time and shader clock of one batch launch, from a -DMCK_TRACE=1
build (make variants VARIANTS="trace:-DMCK_TRACE=1").

Each wave stamps the wall clock (100 MHz) and the shader-clock counter
(clock64) at entry and exit, and its XCC_ID at entry.  Per XCD this prints the
waves it ran, their mean/max end (us after the first entry) and the clock the
XCD ran at over its waves' lives (d clock64 / d wall).  Question it answers:
is the static split's tail (C2: per-XCD mean ends 33-40 us,
profiles/r02/tail_trace_c2_static.json) an XCD running a slower shader clock
(then the kernel is partly clock-bound and fewer instructions per byte move
it), or an XCD getting less memory bandwidth at the same clock?

usage: xcd_clock.py CONFIG[,CONFIG...] [--launches N] [--out FILE]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from mercury_amd import gpu as G  # noqa: E402
from ab_variants import SHAPES, load  # noqa: E402

NW = 16384  # kTraceWaves
TICK_US = 0.01


def run(lib, cfg, launches):
    method, count, length, seed = SHAPES[cfg]
    assert length is not None, "fixed-stride configs only"
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    o = torch.empty(count, dtype=torch.int32 if method == "crc32c" else torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert lib.mchecksum_gpu_prepare(method.encode()) == 0
    rows = []
    for it in range(launches):
        wall = np.zeros(3 * NW, dtype=np.uint64)
        clk = np.zeros(2 * NW, dtype=np.uint64)
        xcc = np.zeros(NW, dtype=np.uint32)
        # (every launch of a config has the same grid: each wave rewrites its own stamps)
        rc = lib.mchecksum_gpu_checksum_fixed(method.encode(), data.data_ptr(), length, length, count, o.data_ptr(), s)
        assert rc == 0
        torch.cuda.synchronize()
        assert lib.mck_debug_trace_read(wall.ctypes.data, wall.nbytes) == 0
        assert lib.mck_debug_trace_clk_read(clk.ctypes.data, clk.nbytes) == 0
        assert lib.mck_debug_trace_xcc_read(xcc.ctypes.data, xcc.nbytes) == 0
        w = wall.reshape(-1, 3).astype(np.int64)
        c = clk.reshape(-1, 2).astype(np.int64)
        live = (w[:, 0] > 0) & (w[:, 2] > w[:, 0]) & (c[:, 1] > c[:, 0])
        w, c, x = w[live], c[live], xcc[live]
        t0 = w[:, 0].min()
        end = (w[:, 2] - t0) * TICK_US
        per = {}
        for k in sorted(set(x.tolist())):
            m = x == k
            mhz = (c[m, 1] - c[m, 0]).sum() / ((w[m, 2] - w[m, 0]).sum() * TICK_US)
            per[int(k)] = {"waves": int(m.sum()), "end_mean_us": round(float(end[m].mean()), 2),
                           "end_max_us": round(float(end[m].max()), 2), "sclk_mhz": round(float(mhz), 0)}
        rows.append({"launch": it, "waves": int(live.sum()), "end_max_us": round(float(end.max()), 2), "xcd": per})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs")
    ap.add_argument("--launches", type=int, default=12)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    lib = load(os.path.join(ROOT, "build", "variants", os.environ.get("TRACE_LIB", "libmchecksum_trace.so")))
    for n in ("mck_debug_trace_read", "mck_debug_trace_clk_read", "mck_debug_trace_xcc_read"):
        getattr(lib, n).argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    out = {}
    for cfg in args.configs.split(","):
        rows = run(lib, cfg, args.launches)
        out[cfg] = rows
        for r in rows[2:]:
            xs = r["xcd"]
            print(cfg, r["launch"], "end_max", r["end_max_us"], " ".join(
                f"x{k}:{v['end_mean_us']}/{v['sclk_mhz']:.0f}MHz" for k, v in xs.items()), flush=True)
        # correlation of per-XCD mean end with per-XCD clock over the steady launches
        e = np.array([[v["end_mean_us"] for v in r["xcd"].values()] for r in rows[2:]]).ravel()
        f = np.array([[v["sclk_mhz"] for v in r["xcd"].values()] for r in rows[2:]]).ravel()
        if len(e) > 2 and e.std() > 0 and f.std() > 0:
            print(cfg, "corr(end_mean, sclk) over XCDs x launches:", round(float(np.corrcoef(e, f)[0, 1]), 3))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
