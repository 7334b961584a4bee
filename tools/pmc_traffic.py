#!/usr/bin/env python3
"""HBM traffic per launch of the dominant kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), corrected as
/opt/skills/guides/MI355X_MICROARCH.md sec. HBM prescribes: both counters are
in KiB; FETCH_SIZE reads exactly half the bytes of a wide coalesced streaming
read on gfx950, so it is doubled.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTRING OUT_JSON [alg_bytes [dispatches_per_call [last]]]
(dispatches_per_call: kernels matching the substring per API call, e.g. 3 for
the segments path: scan + two chunk passes; last: use only the last N matching
dispatches -- the timed calls, not a config's setup launches)
"""
import csv
import glob
import json
import sys


def read(d, counter, ksub):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter or ksub not in row.get("Kernel_Name", ""):
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return [vals[k] for k in sorted(vals, key=lambda k: int(k) if str(k).isdigit() else str(k))]


def main():
    fdir, wdir, ksub, out = sys.argv[1:5]
    alg = float(sys.argv[5]) if len(sys.argv) > 5 else None
    per_call = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    last = int(sys.argv[7]) if len(sys.argv) > 7 else 0
    f = read(fdir, "FETCH_SIZE", ksub)
    w = read(wdir, "WRITE_SIZE", ksub)
    if last:
        f, w = f[-last:], w[-last:]
    if not f or not w:
        raise SystemExit(f"no counter rows for {ksub!r}: fetch={len(f)} write={len(w)}")
    fetch_b = 2 * 1024 * sum(f) / len(f) * per_call
    write_b = 1024 * sum(w) / len(w) * per_call
    res = {"kernel": ksub, "dispatches": {"fetch": len(f), "write": len(w)}, "dispatches_per_call": per_call,
           "fetch_size_kib_raw_mean": sum(f) / len(f), "write_size_kib_mean": sum(w) / len(w),
           "hbm_read_bytes_per_launch": fetch_b, "hbm_write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 x1024, WRITE_SIZE x1024 (MI355X_MICROARCH.md HBM section)"}
    if alg:
        res["algorithmic_bytes_per_launch"] = alg
        res["traffic_over_algorithmic"] = (fetch_b + write_b) / alg
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
