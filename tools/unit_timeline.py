#!/usr/bin/env python3
"""DIAGNOSTIC: completion timeline of one headline launch (65536 x 64 KiB
CRC-32C on the work queue) taken after 40 back-to-back warm-up launches, from
a -DMCK_TRACE=1 build (make variants VARIANTS="trace:-DMCK_TRACE=1").  Bins
unit completions in 10 us steps, in total and per XCD (blockIdx % 8), so the
end of the launch shows whether bandwidth falls off on every XCD together or
XCD by XCD."""
import ctypes, json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_variants import SHAPES, load  # noqa: E402

TICK_US = 0.01  # wall_clock64: 100 MHz
BIN_US = 10.0


def main():
    lib = load(os.path.join(ROOT, "build", "variants", "libmchecksum_trace.so"))
    lib.mck_debug_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.mck_debug_units_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    method, count, length, seed = SHAPES["metric"]
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    o = torch.empty(count, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert lib.mchecksum_gpu_prepare(method.encode()) == 0
    runs = []
    for rep in range(3):
        for _ in range(41):  # 40 warm-up launches back to back, the 41st is traced
            assert lib.mchecksum_gpu_checksum_fixed(method.encode(), data.data_ptr(), length, length, count,
                                                    o.data_ptr(), s) == 0
        torch.cuda.synchronize()
        w = np.zeros(3 * 16384, dtype=np.uint64)
        u = np.zeros(1 << 17, dtype=np.uint64)
        assert lib.mck_debug_trace_read(w.ctypes.data, w.nbytes) == 0
        assert lib.mck_debug_units_read(u.ctypes.data, u.nbytes) == 0
        w = w.reshape(-1, 3).astype(np.int64)
        w = w[w[:, 2] > 0]
        t0 = int(w[:, 0].min())
        u = u[:count]
        xcd = (u >> np.uint64(60)).astype(np.int64)
        t = ((u & np.uint64((1 << 60) - 1)).astype(np.int64) - t0) * TICK_US
        end = float(t.max())
        nb = int(end // BIN_US) + 1
        tot = np.bincount((t // BIN_US).astype(np.int64), minlength=nb)
        gbs = tot * length / (BIN_US * 1e-6) / 1e9
        per = [np.bincount((t[xcd == x] // BIN_US).astype(np.int64), minlength=nb) * length / (BIN_US * 1e-6) / 1e9
               for x in range(8)]
        last_unit_per_xcd = [round(float(t[xcd == x].max()), 1) for x in range(8)]
        units_per_xcd = [int((xcd == x).sum()) for x in range(8)]
        k = 12  # the last 120 us
        r = {"end_us": round(end, 1), "steady_GBps": round(float(np.median(gbs[5:nb - k])), 0),
             "last_bins_GBps": [round(float(v)) for v in gbs[-k:]],
             "last_bins_GBps_per_xcd": [[round(float(v)) for v in p[-k:]] for p in per],
             "last_unit_per_xcd_us": last_unit_per_xcd, "units_per_xcd": units_per_xcd,
             "first_bins_GBps": [round(float(v)) for v in gbs[:6]]}
        print(json.dumps(r), flush=True)
        runs.append(r)
    json.dump(runs, open(os.path.join(ROOT, "gpurun_out", "unit_timeline.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
