#!/usr/bin/env python3
"""A/B the batch-kernel variants built by `make variants` in ONE process,
interleaved round by round (cdna_hip_programming.md sec. 5.4 rule 24).

Every variant must produce the same CRCs as the default library; the script
prints per-variant median/min kernel time and achieved HBM GB/s.
"""
import argparse
import ctypes
import glob
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402

SHAPES = {
    "metric": ("crc32c", 65536, 65536, 0x4D43310000000005),
    "c2": ("crc32c", 65536, 4096, 0x4D43310000000002),
    # lanes-per-payload policy (choose_log2g) checks: other fixed payload sizes
    "f1k": ("crc32c", 262144, 1024, 0x4D43310000000002),
    "f2k": ("crc32c", 131072, 2048, 0x4D43310000000002),
    "f8k": ("crc32c", 65536, 8192, 0x4D43310000000002),
    "f16k": ("crc32c", 65536, 16384, 0x4D43310000000002),
    "s8192": ("crc32c", 8192, 4096, 0x4D43310000000002),     # 32 MiB: just past the light layout
    "s2048": ("crc32c", 2048, 4096, 0x4D43310000000002),
    "g4k": ("crc64", 65536, 4096, 0x4D43310000000003),
    "g16k": ("crc64", 32768, 16384, 0x4D43310000000003),
    "g64k": ("crc64", 16384, 65536, 0x4D43310000000003),
    "c3": ("crc64", 8192, 1 << 20, 0x4D43310000000003),
    "m1": ("crc64", 256, 1 << 20, 0x4D43310000000003),     # 256 MiB: 64-lane CRC-64 payloads, not split
    "c4": ("crc32c", 262144, None, 0x4D43310000000004),   # offsets table, U[64 B, 64 KiB]
    "c4_64": ("crc64", 262144, None, 0x4D43310000000004),
    "seg": ("crc64", 8192, "seg", 0x4D43310000000003),      # bench.py's segments layout
    "seg32": ("crc32c", 8192, "seg", 0x4D43310000000003),   # the same layout, CRC-32C
    # small batches (per-call latency; the light layout up to 16 MiB)
    "s1": ("crc32c", 1, 4096, 0x4D43310000000002),
    "s64": ("crc32c", 64, 4096, 0x4D43310000000002),
    "s1024": ("crc32c", 1024, 4096, 0x4D43310000000002),
    "s4096": ("crc32c", 4096, 4096, 0x4D43310000000002),
    "s1_64k": ("crc32c", 1, 65536, 0x4D43310000000002),
    "c64s1": ("crc64", 1, 4096, 0x4D43310000000003),
    "c64s1024": ("crc64", 1024, 4096, 0x4D43310000000003),
}


def reload_settings(L):
    """The library reads its MCHECKSUM_* settings once; re-read them (builds
    from before round 6 read them on every call and have no such entry)."""
    f = getattr(L, "mchecksum_gpu_reload_settings", None)
    if f is not None:
        f()


def load(path):
    L = ctypes.CDLL(path)
    c = ctypes
    L.mchecksum_gpu_prepare.argtypes = [c.c_char_p]
    L.mchecksum_gpu_checksum_fixed.argtypes = [c.c_char_p, c.c_void_p, c.c_size_t, c.c_size_t, c.c_size_t,
                                               c.c_void_p, c.c_void_p]
    L.mchecksum_gpu_checksum_offsets.argtypes = [c.c_char_p, c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p,
                                                 c.c_void_p]
    L.mchecksum_gpu_checksum_segments.argtypes = [c.c_char_p, c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p,
                                                  c.c_size_t, c.c_void_p, c.c_size_t, c.c_void_p, c.c_void_p]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="metric")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--variants", nargs="*", default=None)
    ap.add_argument("--env", nargs="*", default=[],
                    help="extra pseudo-variants of the default library: NAME=VAR=VALUE (env set around its calls)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--nocheck", nargs="*", default=[],
                    help="timing-only experiment variants whose CRCs are not compared with the default library's")
    ap.add_argument("--rotate", type=int, default=1,
                    help="fixed shapes: launch k reads copy k %% R of R equal batches at distinct addresses "
                         "(cold lines: no launch re-reads what the last one left in the Infinity Cache)")
    ap.add_argument("--series", action="store_true",
                    help="one event pair around each round's back-to-back launches (bench.py's timing: the "
                         "boundaries between launches count) instead of one pair per launch")
    args = ap.parse_args()

    paths = sorted(glob.glob(os.path.join(ROOT, "build", "variants", "libmchecksum_*.so")))
    if args.variants:
        paths = [p for p in paths if os.path.basename(p)[len("libmchecksum_"):-3] in args.variants]
    names = [os.path.basename(p)[len("libmchecksum_"):-3] for p in paths]
    libs = [load(p) for p in paths]
    envs = [None] * len(libs)
    for spec in args.env:  # NAME=VAR=VALUE[@variant]: a library run with VAR=VALUE set around its calls
        spec, _, base = spec.partition("@")
        nm, var, val = spec.split("=", 2)
        names.append(nm)
        libs.append(load(os.path.join(ROOT, "build", "variants", f"libmchecksum_{base}.so") if base
                         else os.path.join(ROOT, "mercury_amd", "lib", "libmchecksum.so")))
        envs.append((var, val))

    results = {}
    configs = args.config.split(",")
    for cfg in configs:
        method, count, length, seed = SHAPES[cfg]
        offs = seg = None
        if length == "seg":
            from mercury_amd.workload import segment_slots
            nbytes, slen = count << 20, (1 << 20) // 4
            data = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
            G.fill_splitmix(data, seed)
            slots = segment_slots(seed, count * 4)
            seg = G.SegmentBatch([data[int(q) * slen:(int(q) + 1) * slen] for q in slots],
                                 np.arange(0, count * 4 + 1, 4))
            seg.work = torch.empty(2 * seg.work.numel() + (1 << 17), dtype=torch.int64, device="cuda")  # room for any variant
            ref = seg.checksum(method)
        elif length is None:
            from mercury_amd.workload import varlen_offsets
            off_h = varlen_offsets(seed, count)
            nbytes = int(off_h[-1])
            data = torch.empty(nbytes + 64, dtype=torch.uint8, device="cuda")
            offs = torch.from_numpy(off_h.astype(np.int64)).cuda()
            G.fill_splitmix(data, seed)
            ref = G.checksum_offsets(method, data, offs, offsets_host=off_h)
        else:
            nbytes = count * length
            copies = [torch.empty(count * length + 64, dtype=torch.uint8, device="cuda") for _ in range(args.rotate)]
            for d in copies:
                G.fill_splitmix(d, seed)
            data = copies[0]
            ref = G.checksum_fixed(method, data, length, count=count)
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream()
        h = stream.cuda_stream
        outs = [torch.empty_like(ref) for _ in libs]
        for L in libs:
            assert L.mchecksum_gpu_prepare(method.encode()) == 0
        times = {n: [] for n in names}
        for r in range(args.rounds + 1):
            for n, L, o, e in zip(names, libs, outs, envs):
                if e:
                    os.environ[e[0]] = e[1]
                    reload_settings(L)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(1 if args.series else args.iters)]
                for k in range(args.iters):
                    a, b = evs[0 if args.series else k]
                    if not args.series or k == 0:
                        a.record(stream)
                    if seg is not None:
                        mb, ns = seg.meta.data_ptr(), seg.nseg
                        rc = L.mchecksum_gpu_checksum_segments(method.encode(), mb, mb + 8 * ns, ns, mb + 16 * ns, seg.nobj,
                                                               seg.work.data_ptr(), seg.work.numel() * 8, o.data_ptr(), h)
                    elif offs is None:
                        d = copies[k % len(copies)]
                        rc = L.mchecksum_gpu_checksum_fixed(method.encode(), d.data_ptr(), length, length, count,
                                                            o.data_ptr(), h)
                    else:
                        rc = L.mchecksum_gpu_checksum_offsets(method.encode(), data.data_ptr(), offs.data_ptr(),
                                                              count, o.data_ptr(), h)
                    if not args.series or k == args.iters - 1:
                        b.record(stream)
                    assert rc == 0
                torch.cuda.synchronize()
                if e:
                    del os.environ[e[0]]
                    reload_settings(L)
                if r > 0:  # round 0 = warm-up
                    times[n] += [a.elapsed_time(b) / (args.iters if args.series else 1) for a, b in evs]
        for n, o in zip(names, outs):
            if n in args.nocheck:
                continue
            assert torch.equal(o, ref), f"variant {n} differs from the default library"
        res = {}
        for n in names:
            t = np.array(times[n])
            res[n] = {"median_ms": float(np.median(t)), "min_ms": float(t.min()),
                      "GBs_median": nbytes / (np.median(t) * 1e-3) / 1e9, "GBs_best": nbytes / (t.min() * 1e-3) / 1e9}
            print(f"{cfg:7s} {n:10s} median {res[n]['median_ms']:.4f} ms  min {res[n]['min_ms']:.4f} ms  "
                  f"{res[n]['GBs_median']:.0f} GB/s (best {res[n]['GBs_best']:.0f})", flush=True)
        results[cfg] = res
        del data
        copies = None
        torch.cuda.empty_cache()
    if args.out:
        json.dump(results, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
