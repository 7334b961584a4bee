#!/usr/bin/env python3
"""Per-wave timeline of one batch launch from a -DMCK_TRACE=1 build
(make variants VARIANTS="trace:-DMCK_TRACE=1"): when waves enter, finish the
LDS fill and exit, relative to the first entry (wall_clock64, 100 MHz).
Shows the launch ramp and the tail that static payload assignment leaves.
ROTATE=R: R copies of each fixed batch, read in turn (cold lines, as
bench.py --rotate), back-to-back launches with the traced one last."""
import ctypes, json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_variants import SHAPES, load  # noqa: E402

TICK_US = 0.01  # 100 MHz


def main():
    lib = load(os.path.join(ROOT, "build", "variants", os.environ.get("TRACE_LIB", "libmchecksum_trace.so")))
    lib.mck_debug_trace_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.mck_debug_qwave_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    out = {}
    for cfg in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["metric", "c2", "c4"]):
        method, count, length, seed = SHAPES[cfg]
        if length is None:
            from mercury_amd.workload import varlen_offsets
            off_h = varlen_offsets(seed, count)
            data = torch.empty(int(off_h[-1]) + 64, dtype=torch.uint8, device="cuda")
            offs = torch.from_numpy(off_h.astype(np.int64)).cuda()
        else:
            data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
            offs = None
        G.fill_splitmix(data, seed)
        rot = int(os.environ.get("ROTATE", "1")) if offs is None else 1
        copies = [data] + [data.clone() for _ in range(rot - 1)]
        o = torch.empty(count, dtype=torch.int32 if method == "crc32c" else torch.int64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        assert lib.mchecksum_gpu_prepare(method.encode()) == 0
        res = []
        for it in range(12):
            buf = np.zeros(3 * 16384, dtype=np.uint64)
            lib.mck_debug_trace_read(buf.ctypes.data, buf.nbytes)  # (stale values are masked below)
            torch.cuda.synchronize()
            for b in range(rot - 1):  # the launches before the traced one, back to back
                assert lib.mchecksum_gpu_checksum_fixed(method.encode(), copies[b].data_ptr(), length, length, count,
                                                        o.data_ptr(), s) == 0
            if offs is None:
                rc = lib.mchecksum_gpu_checksum_fixed(method.encode(), copies[-1].data_ptr(), length, length, count,
                                                      o.data_ptr(), s)
            else:
                rc = lib.mchecksum_gpu_checksum_offsets(method.encode(), data.data_ptr(), offs.data_ptr(), count, o.data_ptr(), s)
            assert rc == 0
            torch.cuda.synchronize()
            assert lib.mck_debug_trace_read(buf.ctypes.data, buf.nbytes) == 0
            qraw = np.zeros(6 * 16384, dtype=np.uint64)
            lib.mck_debug_qwave_read(qraw.ctypes.data, qraw.nbytes)
            qw = qraw[:4 * 16384].reshape(-1, 4).astype(np.float64)
            qu = qraw[4 * 16384:].reshape(-1, 2).astype(np.float64)
            t = buf.reshape(-1, 3).astype(np.int64)
            t = t[t[:, 2] > 0]
            t0 = t[:, 0].min()
            ent, fill, end = (t[:, 0] - t0) * TICK_US, (t[:, 1] - t[:, 0]) * TICK_US, (t[:, 2] - t0) * TICK_US
            r = {"waves": int(len(t)), "entry_p50_us": float(np.median(ent)), "entry_max_us": float(ent.max()),
                 "fill_p50_us": float(np.median(fill)), "fill_max_us": float(fill.max()),
                 "end_p10_us": float(np.percentile(end, 10)), "end_p50_us": float(np.median(end)),
                 "end_p90_us": float(np.percentile(end, 90)), "end_max_us": float(end.max())}
            nb = len(t) // 16 if len(t) >= 16 else 1
            xcd = [float(np.mean(end[np.arange(len(t)) // 16 % 8 == x])) for x in range(8)] if len(t) >= 128 else []
            r["end_mean_per_xcd_us"] = [round(v, 1) for v in xcd]
            act = qw[:, 0] > 0
            r["fetches"] = float(qw[:, 0].sum())
            r["fetch_mean_us"] = float(qw[:, 1].sum() / max(1.0, qw[:, 0].sum()) * TICK_US)
            r["fetch_max_us"] = float(qw[:, 2].max() * TICK_US)
            r["wave_wait_mean_us"] = float(qw[:, 3].mean() * TICK_US)
            r["wave_wait_max_us"] = float(qw[:, 3].max() * TICK_US)
            r["units_total"] = float(qu[:, 0].sum())
            r["units_per_wave_min_max"] = [float(qu[:len(t), 0].min()), float(qu[:len(t), 0].max())]
            r["unit_us"] = float(qu[:, 1].sum() / max(1.0, qu[:, 0].sum()) * TICK_US)
            if it >= 2:
                res.append(r)
        keys = [k for k in res[0] if k not in ("end_mean_per_xcd_us", "waves", "units_per_wave_min_max")]
        med = {k: round(float(np.median([r[k] for r in res])), 2) for k in keys}
        med["waves"] = res[0]["waves"]
        med["units_per_wave_min_max(last)"] = res[-1].get("units_per_wave_min_max")
        med["end_mean_per_xcd_us(last)"] = res[-1]["end_mean_per_xcd_us"]
        print(cfg, json.dumps(med), flush=True)
        out[cfg] = med
        del data, copies
        torch.cuda.empty_cache()
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", os.environ.get("TRACE_OUT", "tail_trace.json")), "w"), indent=1)


if __name__ == "__main__":
    main()
