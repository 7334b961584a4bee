#!/usr/bin/env python3
"""End-to-end rate of the checksum path when payloads start in host memory
(NA recv buffers / hg_proc buffers are host memory in Mercury): pinned host ->
H2D -> batch CRC kernel -> D2H of the CRCs, double-buffered so copies overlap
the kernel on separate HIP streams.  Reports the overlapped rate next to the
H2D copy alone (the PCIe bound) and the kernel alone: the median of --reps
timed runs (and min/max), after one untimed run.  The CRCs that came back to
the host are checked against the CPU oracle (oracle/, test infrastructure:
this diagnostic is a checker here) on sampled payloads, and against a
device-resident run on all of them.  Written into DESIGN.md; never the bench
`value`.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-mib", type=int, default=4096)
    ap.add_argument("--chunk-mib", type=int, default=128)
    ap.add_argument("--length", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    length = args.length
    chunk = args.chunk_mib << 20
    nchunks = (args.total_mib << 20) // chunk
    per_chunk = chunk // length
    host = torch.empty(nchunks * chunk, dtype=torch.uint8, pin_memory=True)
    # fill host bytes via the device generator once (content is irrelevant to timing)
    tmp = torch.empty(chunk + 64, dtype=torch.uint8, device="cuda")
    for i in range(nchunks):
        G.fill_splitmix(tmp, 0x4D43310000000005, first_word=i * chunk // 8)
        host[i * chunk:(i + 1) * chunk].copy_(tmp[:chunk])
    torch.cuda.synchronize()
    G.prepare("crc32c")
    dbuf = [torch.empty(chunk + 64, dtype=torch.uint8, device="cuda") for _ in range(2)]
    dout = [torch.empty(per_chunk, dtype=torch.int32, device="cuda") for _ in range(2)]
    hout = torch.empty(nchunks * per_chunk, dtype=torch.int32, pin_memory=True)
    s_copy, s_comp = torch.cuda.Stream(), torch.cuda.Stream()

    def h2d_only():
        for i in range(nchunks):
            with torch.cuda.stream(s_copy):
                dbuf[i % 2][:chunk].copy_(host[i * chunk:(i + 1) * chunk], non_blocking=True)

    def kernel_only():
        for i in range(nchunks):
            G.checksum_fixed("crc32c", dbuf[i % 2], length, count=per_chunk, out=dout[i % 2], stream=s_comp)

    def pipelined():
        copied = [torch.cuda.Event() for _ in range(2)]
        done = [torch.cuda.Event() for _ in range(2)]
        for e in done:
            e.record(s_comp)
        for i in range(nchunks):
            b = i % 2
            s_copy.wait_event(done[b])
            with torch.cuda.stream(s_copy):
                dbuf[b][:chunk].copy_(host[i * chunk:(i + 1) * chunk], non_blocking=True)
                copied[b].record(s_copy)
            s_comp.wait_event(copied[b])
            G.checksum_fixed("crc32c", dbuf[b], length, count=per_chunk, out=dout[b], stream=s_comp)
            with torch.cuda.stream(s_comp):
                hout[i * per_chunk:(i + 1) * per_chunk].copy_(dout[b], non_blocking=True)
            done[b].record(s_comp)

    res = {}
    for name, fn in (("h2d_only", h2d_only), ("kernel_only", kernel_only), ("pipelined_e2e", pipelined)):
        fn()
        torch.cuda.synchronize()
        laps = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            laps.append(time.perf_counter() - t0)
        laps.sort()
        med = laps[len(laps) // 2]
        res[name] = {"median_s": med, "min_s": laps[0], "max_s": laps[-1], "reps": len(laps),
                     "GB_s_median": nchunks * chunk / med / 1e9, "GiB_s_median": nchunks * chunk / med / 2**30}
    # parity of the e2e result against a device-resident run
    ref = torch.empty(nchunks * per_chunk, dtype=torch.int32, device="cuda")
    for i in range(nchunks):
        dbuf[0][:chunk].copy_(host[i * chunk:(i + 1) * chunk])
        G.checksum_fixed("crc32c", dbuf[0], length, count=per_chunk, out=ref[i * per_chunk:(i + 1) * per_chunk])
    torch.cuda.synchronize()
    res["e2e_matches_device_resident"] = bool(torch.equal(ref.cpu(), hout))
    # ... and the oracle on sampled payloads (first, last, 62 random)
    import numpy as np
    from oracle import oracle as O
    got = hout.numpy().view(np.uint32)
    idx = np.unique(np.concatenate([[0, len(got) - 1], np.random.default_rng(7).integers(0, len(got), 62)]))
    hb = host.numpy()
    bad = sum(int(got[i]) != O.crc("crc32c", hb[i * length:(i + 1) * length]) for i in idx)
    res["oracle_check"] = f"{len(idx) - bad}/{len(idx)} sampled payloads equal the oracle"
    res["config"] = {"total_bytes": nchunks * chunk, "chunk_bytes": chunk, "payload_bytes": length,
                     "pcie_spec_GB_s": 63.0}
    print(json.dumps(res))
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
