#!/usr/bin/env python3
"""Do consecutive headline launches on different streams overlap on the GPU?

Runs the headline batch (65536 x 64 KiB CRC-32C, device-resident) K times,
launch i on stream i % S, with S pool streams (none of them the default
stream), and prints the wall time per launch.  Run under
`rocprofv3 --kernel-trace` and read the trace with --analyze: for each launch,
the gap (negative = overlap) between its start and the previous launch's end.

usage: overlap_probe.py [--streams S] [--steps K] [--warmup W]
       overlap_probe.py --analyze KERNEL_TRACE.csv
"""
import argparse
import csv
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def analyze(path, key="crc32c_batch_kernel", group=0):
    rows = [r for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if group:  # gap statistics per consecutive group of dispatches (one per probe mode)
        for g in range(0, len(rows) - group + 1, group):
            part = rows[g:g + group]
            gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(part, part[1:])]
            dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in part]
            print(json.dumps({"group": g // group, "dur_median_us": round(statistics.median(dur), 2),
                              "gap_median_us": round(statistics.median(gaps), 2), "gap_min_us": round(min(gaps), 2)}))
        return
    s = [int(r["Start_Timestamp"]) for r in rows]
    e = [int(r["End_Timestamp"]) for r in rows]
    gaps = [(s[i] - e[i - 1]) / 1e3 for i in range(1, len(rows))]
    dur = [(e[i] - s[i]) / 1e3 for i in range(len(rows))]
    span = (e[-1] - s[0]) / 1e3
    out = {"dispatches": len(rows), "queues": sorted({r.get("Queue_Id", "?") for r in rows}),
           "dur_mean_us": round(statistics.mean(dur), 2), "gap_mean_us": round(statistics.mean(gaps), 2),
           "gap_min_us": round(min(gaps), 2), "gap_max_us": round(max(gaps), 2),
           "span_per_launch_us (last 20)": round((e[-1] - s[-20]) / 1e3 / 20, 2) if len(rows) >= 20 else None,
           "span_us": round(span, 1)}
    json.dump(out, sys.stdout, indent=1)
    print()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--analyze")
    ap.add_argument("--kernel", default="crc32c_batch_kernel")
    ap.add_argument("--group", type=int, default=0)
    args = ap.parse_args()
    if args.analyze:
        return analyze(args.analyze, args.kernel, args.group)
    import torch
    from mercury_amd import gpu as G
    n, length = 65536, 65536
    data = torch.empty(n * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, 0x4D43310000000005)
    G.prepare("crc32c")
    streams = [torch.cuda.Stream() for _ in range(args.streams)]
    outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in streams]
    print("stream handles", [hex(s.cuda_stream) for s in streams], file=sys.stderr)

    def run(k):
        for i in range(k):
            with torch.cuda.stream(streams[i % len(streams)]):
                G.checksum_fixed("crc32c", data, length, count=n, out=outs[i % len(streams)])

    run(args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    ref = outs[0].clone()
    same = all(torch.equal(o, ref) for o in outs)
    print(json.dumps({"streams": args.streams, "ms_per_launch": round(dt * 1e3, 4),
                      "of_8TBs": round((n * length + 4 * n) / dt / 8e12, 4), "outputs_equal": same}))


if __name__ == "__main__":
    main()
