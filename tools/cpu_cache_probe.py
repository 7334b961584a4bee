#!/usr/bin/env python3
"""Host CPU crc32c rate (oracle SSE4.2 path, 1 and 16 threads) over C4-mix
samples of 64 MiB .. 4 GiB: is bench.py's 256 MiB cpu_baseline sample
inflated by the host's L3?  (Output: profiles/r03/cpu_cache_probe.txt.)"""
import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
from oracle import oracle as O
from mercury_amd.workload import varlen_offsets
full = varlen_offsets(0x4D43310000000004, 262144)
for mib in (64, 256, 1024, 4096):
    n = int(np.searchsorted(full, np.uint64(mib << 20)))
    off = np.ascontiguousarray(full[:n + 1]); nb = int(off[-1])
    host = O.splitmix_bytes(nb, 4)
    for th in (1, 16):
        O.batch_offsets("crc32c", host, off, variant="sse42", nthreads=th)
        laps = []
        for _ in range(5 if mib < 4096 else 2):
            t = time.perf_counter(); O.batch_offsets("crc32c", host, off, variant="sse42", nthreads=th); laps.append(time.perf_counter() - t)
        print(mib, "MiB", th, "threads", round(nb / min(laps) / 1e9, 1), "GB/s best", round(nb / float(np.median(laps)) / 1e9, 1), "median", flush=True)
