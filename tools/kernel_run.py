#!/usr/bin/env python3
"""DIAGNOSTIC: run one config's batch kernel N times (for rocprofv3 --pmc passes)."""
import argparse, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from mercury_amd import gpu as G
from tools_shapes import SHAPES
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--iters", type=int, default=5)
# fixed layouts: launch i reads copy i % R of R equal batches at distinct
# addresses (bench.py --rotate: C2's 256 MiB is Infinity-Cache sized)
ap.add_argument("--rotate", type=int, default=1)
a = ap.parse_args()
method, count, length, seed = SHAPES[a.config]
if a.config == "msgs":  # bench.py's msgs layout: HG header (network-order payload CRC) at 16, payload from 20
    from mercury_amd.workload import varlen_offsets
    off = varlen_offsets(seed, count)
    data = torch.empty(int(off[-1]) + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    inter = np.empty(2 * count + 1, dtype=np.uint64)
    inter[0::2] = off
    inter[1::2] = off[:-1] + np.uint64(20)
    sender = G.checksum_offsets(method, data, torch.from_numpy(inter.astype(np.int64)).cuda())
    offs = torch.from_numpy(off.astype(np.int64)).cuda()
    crc = sender[1::2].to(torch.int64) & 0xFFFFFFFF
    for k in range(4):
        data[offs[:-1] + 16 + k] = ((crc >> (24 - 8 * k)) & 0xFF).to(torch.uint8)
    status = torch.empty(count, dtype=torch.uint8, device="cuda")
    mism = torch.zeros(1, dtype=torch.int32, device="cuda")
    run = lambda: G.verify_messages(data, offs, status=status, mismatches=mism)
elif a.config == "xdr":  # bench.py's xdr layout: hg_perf_proc_iovec messages in XDR mode
    import bench
    from mercury_amd.workload import varlen_lengths
    off = bench.xdr_offsets(seed, count)
    lens = torch.from_numpy(varlen_lengths(seed, count).astype(np.int64)).cuda()
    data = torch.empty(int(off[-1]) + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    offs = torch.from_numpy(off.astype(np.int64)).cuda()
    for k in range(4):
        data[offs[:-1] + k] = ((lens >> (24 - 8 * k)) & 0xFF).to(torch.uint8)
    xout = torch.empty(count, dtype=torch.int32, device="cuda")
    run = lambda: G.checksum_xdr(method, data, offs, bench.XDR_IOVEC, out=xout)
elif a.config == "seg":  # bench.py's segments layout: 4 scattered 256 KiB segments per 1 MiB object
    from mercury_amd.workload import segment_slots
    slen = length // 4
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    slots = segment_slots(seed, count * 4)
    batch = G.SegmentBatch([data[int(q) * slen:(int(q) + 1) * slen] for q in slots], np.arange(0, count * 4 + 1, 4))
    sout = torch.empty(count, dtype=torch.int64, device="cuda")
    run = lambda: batch.checksum(method, out=sout)
elif length is None:
    from mercury_amd.workload import varlen_offsets
    off = varlen_offsets(seed, count)
    data = torch.empty(int(off[-1]) + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, seed)
    offs = torch.from_numpy(off.astype(np.int64)).cuda()
    run = lambda: G.checksum_offsets(method, data, offs)
else:
    datas = [torch.empty(count * length + 64, dtype=torch.uint8, device="cuda") for _ in range(a.rotate)]
    for d in datas:
        G.fill_splitmix(d, seed)
    it = [0]

    def run():
        G.checksum_fixed(method, datas[it[0] % len(datas)], length, count=count)
        it[0] += 1
for _ in range(a.iters):
    run()
torch.cuda.synchronize()
print("ok")
