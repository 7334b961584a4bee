#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per kernel over dispatches (skipping the
first, cold one).  usage: pmc_summary.py DIR [DIR...]
PMC_KERNELS (comma-separated substrings, default batch_kernel) picks the kernels."""
import csv, glob, os, sys
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        per = defaultdict(lambda: defaultdict(float))
        for r in rows:
            per[(r["Kernel_Name"], r.get("Dispatch_Id"))][r["Counter_Name"]] += float(r["Counter_Value"])
        by_k = defaultdict(list)
        for (k, did), c in per.items():
            by_k[k].append((int(did), c))
        for k, lst in by_k.items():
            lst.sort()
            for did, c in lst[1:] or lst:
                for n, v in c.items():
                    vals[k][n].append(v)
for k, c in vals.items():
    if not any(s in k for s in os.environ.get("PMC_KERNELS", "batch_kernel").split(",")):
        continue
    print(k[:90])
    for n in sorted(c):
        v = c[n]
        print(f"   {n:28s} {sum(v)/len(v):.4e}  (n={len(v)})")
