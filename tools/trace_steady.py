#!/usr/bin/env python3
"""Per-launch durations of one kernel from a rocprofv3 --kernel-trace CSV,
split the way bench.py runs it: the first `warmup` dispatches (DVFS settling,
DESIGN.md sec. 6) and the last `steps` ones (the timed region).  The mean over
the timed dispatches is the rocprof counterpart of bench.py's
roofline.kernel_ms; the --stats summary averages over every dispatch.

usage: trace_steady.py KERNEL_TRACE.csv KERNEL_SUBSTRING WARMUP STEPS [BENCH.json] [--skip N] > out.json

By default the timed region is the kernel's last STEPS dispatches.  With
--skip N it is dispatches [N + WARMUP, N + WARMUP + STEPS) in time order: the
default bench.py line launches the headline's kernel first for the e2e
zero-copy leg (1 + --e2e-reps launches), then for c5_strong, and the
headline's own dispatches come last (the default region); c5_strong's region
is --skip 6 at the default 5 reps (--skip 0 with --no-e2e), and BENCH.json's
c5_strong.kernel_ms is its counterpart.
"""
import csv
import json
import statistics
import sys


def main():
    argv = sys.argv[1:]
    skip = None
    if "--skip" in argv:
        i = argv.index("--skip")
        skip = int(argv[i + 1])
        del argv[i:i + 2]
    path, key, warmup, steps = argv[0], argv[1], int(argv[2]), int(argv[3])
    rows = [r for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    need = warmup + steps + (skip or 0)
    if len(us) < need:
        raise SystemExit(f"{len(us)} dispatches of {key!r}, expected >= {need}")
    if skip is None:
        warm, timed = us[len(us) - steps - warmup:len(us) - steps], us[-steps:]
    else:
        warm, timed = us[skip:skip + warmup], us[skip + warmup:skip + warmup + steps]
    out = {
        "kernel": rows[0]["Kernel_Name"],
        "dispatches": len(us),
        "all_mean_us": round(statistics.mean(us), 2),
        "region": "last" if skip is None else f"skip {skip}",
        "warmup_mean_us": round(statistics.mean(warm), 2) if warmup else None,
        "timed_mean_us": round(statistics.mean(timed), 2),
        "timed_median_us": round(statistics.median(timed), 2),
        "timed_min_us": round(min(timed), 2),
        "timed_max_us": round(max(timed), 2),
    }
    if len(argv) > 4:
        b = json.load(open(argv[4]))
        out["bench_kernel_ms"] = (b["c5_strong"]["kernel_ms"] if skip is not None and "c5_strong" in b
                                  else b["roofline"]["kernel_ms"])
        out["timed_mean_vs_bench"] = round(out["timed_mean_us"] / 1e3 / out["bench_kernel_ms"], 4)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
