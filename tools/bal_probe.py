#!/usr/bin/env python3
"""The balanced static split launch by launch (-DMCK_TRACE=1 build,
make variants VARIANTS="trace:-DMCK_TRACE=1"): for a series of back-to-back
launches of one shape on one stream, the weights each launch used (the slot's
BalBank), each group's measured span, and from the per-wave stamps the mean /
max end per group (blockIdx % 8) and per hardware XCD (XCC_ID) -- first with
the plain split (MCHECKSUM_GPU_BAL=0), then balanced.  Output: JSON lines."""
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

TICK_US = 0.01
ONE = 1 << 24


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n_launch = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    lib = load(os.path.join(ROOT, "build", "variants", os.environ.get("TRACE_LIB", "libmchecksum_trace.so")))
    for f in ("mck_debug_trace_read", "mck_debug_trace_xcc_read"):
        getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.mck_debug_bal_read.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    method, count, length, seed = SHAPES[cfg]
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    ref = G.checksum_fixed(method, data, length, count=count)
    out = torch.empty_like(ref)
    h = torch.cuda.current_stream().cuda_stream
    assert lib.mchecksum_gpu_prepare(method.encode()) == 0
    bank_bytes = 64 + 16 * 512
    seq = 0
    for mode in ("plain", "bal"):
        if mode == "plain":
            os.environ["MCHECKSUM_GPU_BAL"] = "0"
        else:
            os.environ.pop("MCHECKSUM_GPU_BAL", None)
        for it in range(n_launch):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            assert lib.mchecksum_gpu_checksum_fixed(method.encode(), data.data_ptr(), length, length, count,
                                                    out.data_ptr(), h) == 0
            b.record()
            torch.cuda.synchronize()
            assert torch.equal(out, ref), (mode, it)
            st = np.zeros(3 * 16384, dtype=np.uint64)
            xc = np.zeros(16384, dtype=np.uint32)
            assert lib.mck_debug_trace_read(st.ctypes.data, st.nbytes) == 0
            assert lib.mck_debug_trace_xcc_read(xc.ctypes.data, xc.nbytes) == 0
            t = st.reshape(-1, 3).astype(np.int64)
            nw = int(np.count_nonzero(t[:, 2]))
            t, xc = t[:nw], xc[:nw]
            t0 = t[:, 0].min()
            end = (t[:, 2] - t0) * TICK_US
            grp = (np.arange(nw) // 16) % 8
            rec = {"mode": mode, "launch": it, "ms": round(a.elapsed_time(b), 4), "waves": nw,
                   "end_max_us": round(float(end.max()), 2),
                   "group_mean_end": [round(float(end[grp == g].mean()), 1) for g in range(8)],
                   "group_max_end": [round(float(end[grp == g].max()), 1) for g in range(8)],
                   "xcc_mean_end": [round(float(end[xc == x].mean()), 1) if np.any(xc == x) else None for x in range(8)],
                   "group_is_xcc": bool(np.all(xc == grp))}
            if mode == "bal":
                banks = np.zeros(2 * bank_bytes // 8, dtype=np.uint64)
                assert lib.mck_debug_bal_read(0, banks.ctypes.data, banks.nbytes) == 0
                raw = banks.view(np.uint32)
                bank = raw[((seq + 1) & 1) * bank_bytes // 4:][:bank_bytes // 4]  # written by this launch
                w = bank[1:9].astype(np.float64) / ONE
                recs = bank[16:].view(np.uint64).reshape(-1, 2)[:int(bank[0])].astype(np.int64)
                span = [round(float((recs[g::8, 1].max() - recs[g::8, 0].min()) * TICK_US), 1) for g in range(8)]
                rec.update({"grid": int(bank[0]), "weights": [round(float(x) * 8, 3) for x in w], "span_us": span})
                seq += 1
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
