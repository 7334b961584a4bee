#!/usr/bin/env python3
"""Per-launch durations of one kernel from a rocprofv3 --kernel-trace CSV,
split the way bench.py runs it: the first `warmup` dispatches (DVFS settling,
DESIGN.md sec. 6) and the last `steps` ones (the timed region).  The mean over
the timed dispatches is the rocprof counterpart of bench.py's
roofline.kernel_ms; the --stats summary averages over every dispatch.

usage: trace_steady.py KERNEL_TRACE.csv KERNEL_SUBSTRING WARMUP STEPS [BENCH.json] > out.json
"""
import csv
import json
import statistics
import sys


def main():
    path, key, warmup, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = [r for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    if len(us) < warmup + steps:
        raise SystemExit(f"{len(us)} dispatches of {key!r}, expected >= {warmup + steps}")
    timed = us[-steps:]
    out = {
        "kernel": rows[0]["Kernel_Name"],
        "dispatches": len(us),
        "all_mean_us": round(statistics.mean(us), 2),
        "warmup_mean_us": round(statistics.mean(us[:warmup]), 2) if warmup else None,
        "timed_mean_us": round(statistics.mean(timed), 2),
        "timed_median_us": round(statistics.median(timed), 2),
        "timed_min_us": round(min(timed), 2),
        "timed_max_us": round(max(timed), 2),
    }
    if len(sys.argv) > 5:
        b = json.load(open(sys.argv[5]))
        out["bench_kernel_ms"] = b["roofline"]["kernel_ms"]
        out["timed_mean_vs_bench"] = round(out["timed_mean_us"] / 1e3 / b["roofline"]["kernel_ms"], 4)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
